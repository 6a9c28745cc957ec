#!/bin/bash
# GPU box (development only): kbench of library variants, the hot kernel alone
# (trik_hsv_batch_sums) and the full fused step (kbench -s).
#   usage: bash scripts/ab_fused.sh lib...   (dirs under trik-media-sensors-dsp_amd/ab)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fz
K=./scripts/kbench; A=trik-media-sensors-dsp_amd/ab; L=""
for x in "$@"; do L="$L $A/$x/libtrik_hsv.so"; done
timeout -k 10 150 $K -n 50 -r 2 $L > gpurun_out/fz/hot.txt 2>&1 || { cat gpurun_out/fz/hot.txt; exit 3; }
cat gpurun_out/fz/hot.txt
timeout -k 10 150 $K -s -n 50 -r 3 $L > gpurun_out/fz/full.txt 2>&1 || { cat gpurun_out/fz/full.txt; exit 3; }
cat gpurun_out/fz/full.txt
