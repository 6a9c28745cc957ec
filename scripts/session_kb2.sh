#!/bin/bash
# GPU box: hot-kernel parity tests, then kbench A/B (full step, C3 and C4) of ab/ variants
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/kb2; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_chroma.py tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/session_kb.sh "$@"
