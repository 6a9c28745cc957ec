#!/bin/bash
# GPU box: hot-kernel parity tests (incl. AUTO/threads), kbench A/B (C3, C4), and the adversarial table
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/kb3; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_gpu_chroma.py tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_auto.py tests/test_gpu_huefree.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/session_kb.sh "$@" || exit $?
timeout -k 10 600 python scripts/adversarial_ranges.py 4096 > $OUT/adversarial_4096.txt 2>&1; rc=$?; cut -c1-160 $OUT/adversarial_4096.txt | tail -17; exit $rc
