#!/bin/bash
# GPU box (development only): the full fused step (kbench -s) of library
# variants vs the hot kernel alone (kbench).  usage: bash scripts/ab_fused.sh lib...
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fz
K=./scripts/kbench; A=trik-media-sensors-dsp_amd/ab; L=""
for x in "$@"; do L="$L $A/$x/libtrik_hsv.so"; done
timeout -k 10 120 $K -n 50 -r 2 $A/new/libtrik_hsv.so > gpurun_out/fz/hot.txt 2>&1 || exit 3
cat gpurun_out/fz/hot.txt
timeout -k 10 150 $K -s -n 50 -r 3 $L > gpurun_out/fz/full.txt 2>&1 || { cat gpurun_out/fz/full.txt; exit 3; }
cat gpurun_out/fz/full.txt
