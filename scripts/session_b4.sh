#!/bin/bash
# GPU box: blob + operator + C5-shape tests, then blob and auto-range A/B (HEAD vs work tree)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/b4; mkdir -p $OUT
L=trik-media-sensors-dsp_amd
timeout -k 10 700 python -u -m pytest tests/test_gpu_blob.py tests/test_gpu_operator.py tests/test_gpu_auto.py tests/test_gpu_c5.py -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/blob_ab.py $L/ab/blob0/libtrik_hsv.so $L/trik_hsv/libtrik_hsv.so > $OUT/ab_blob.txt 2>&1; rc=$?; cat $OUT/ab_blob.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/blob_ab.py --what range $L/ab/ar0/libtrik_hsv.so $L/trik_hsv/libtrik_hsv.so > $OUT/ab_range.txt 2>&1; rc=$?; cat $OUT/ab_range.txt; exit $rc
