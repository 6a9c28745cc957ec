#!/bin/bash
# GPU box: scripts/session_final2.sh TAG, then the adversarial range-set table
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/session_final2.sh "$1" || exit $?
timeout -k 10 600 python scripts/adversarial_ranges.py 4096 > "gpurun_out/$1/adversarial_4096.txt" 2>&1; rc=$?
tail -20 "gpurun_out/$1/adversarial_4096.txt"; exit $rc
