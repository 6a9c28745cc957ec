#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/b6; mkdir -p $OUT
L=trik-media-sensors-dsp_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_blob.py tests/test_gpu_object_sensor.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/blob_ab.py "$@" > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; exit $rc
