#!/bin/bash
# GPU box (development only): kbench of library variants, the hot kernel alone
# (trik_hsv_batch_sums) and the full fused step (kbench -s) on C3 uniform,
# then the full step on C3 scene frames and on C4.
#   usage: bash scripts/ab_fused.sh lib...   (dirs under trik-media-sensors-dsp_amd/ab)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fz
K=./scripts/kbench; A=trik-media-sensors-dsp_amd/ab; L=""
for x in "$@"; do L="$L $A/$x/libtrik_hsv.so"; done
run() {  # name, kbench args
  local n="$1"; shift
  timeout -k 10 150 $K "$@" $L > "gpurun_out/fz/$n.txt" 2>&1 || { cat "gpurun_out/fz/$n.txt"; exit 3; }
  echo "## $n"; cat "gpurun_out/fz/$n.txt"
}
run hot -n 50 -r 2
run full -s -n 50 -r 3
run full_scene -s -k 1 -n 50 -r 2
run full_c4 -s -f 1024 -w 1280 -h 720 -t 2 -n 50 -r 2
