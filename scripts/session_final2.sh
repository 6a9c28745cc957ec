#!/bin/bash
# GPU box: smoke(), then scripts/session_final.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$1/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/$1/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/session_final.sh "$1"
