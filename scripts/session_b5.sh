#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/b5; mkdir -p $OUT
L=trik-media-sensors-dsp_amd
timeout -k 10 300 python scripts/blob_ab.py $L/trik_hsv/libtrik_hsv.so > $OUT/ab_blob.txt 2>&1; rc=$?; cat $OUT/ab_blob.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/blob_ab.py --what range $L/ab/ar0/libtrik_hsv.so $L/trik_hsv/libtrik_hsv.so > $OUT/ab_range.txt 2>&1; rc=$?; cat $OUT/ab_range.txt; exit $rc
