#!/bin/bash
# GPU box: kbench A/B of chroma-kernel variants (full step, C3 and C4)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/kb; mkdir -p $OUT
L=trik-media-sensors-dsp_amd
LIBS=""; for v in "$@"; do LIBS="$LIBS $L/ab/$v/libtrik_hsv.so"; done
timeout -k 10 240 ./scripts/kbench -s -r 5 $LIBS > $OUT/c3.txt 2>&1; rc=$?; cat $OUT/c3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 ./scripts/kbench -s -r 5 -f 1024 -w 1280 -h 720 -t 2 $LIBS > $OUT/c4.txt 2>&1; rc=$?; cat $OUT/c4.txt; exit $rc
