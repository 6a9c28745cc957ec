#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ar2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_operator.py tests/test_gpu_object_sensor.py tests/test_gpu_threads.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/blob_ab.py --what range trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_operator.py --no-cpu > $OUT/operator.json 2>&1; rc=$?; tail -c 900 $OUT/operator.json; exit $rc
