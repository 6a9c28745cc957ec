#!/bin/bash
# A/B of libtrik_hsv.so variants with the torch-free timer (development only).
# usage (on the GPU box): bash scripts/ab_kbench.sh "kbench flags" lib1 [lib2 ...]
#   libs relative to trik-media-sensors-dsp_amd/ (e.g. ab/base/libtrik_hsv.so)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ab; mkdir -p $OUT
FLAGS="$1"; shift
LIBS=""
for L in "$@"; do LIBS="$LIBS $GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$L"; done
timeout -k 10 240 ./scripts/kbench $FLAGS $LIBS > $OUT/kbench.log 2>&1
rc=$?; cat $OUT/kbench.log; exit $rc
