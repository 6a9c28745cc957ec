#!/bin/bash
# GPU box, round 4: kernel A/Bs then the GPU suite and the driver's bench line.
#   bash scripts/session_r04_ab.sh TAG "kbench runs (flags|libs;...)" "operator-A/B libs" "blob-A/B libs" [pytest selection]
set -u
cd "$GRAFT_REPO_ROOT"; TAG="$1"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ -n "${3:-}" ]; then
  bash scripts/operator_ab.sh "$OUT/op" $3 > "$OUT/operator_ab.txt" 2>&1; rc=$?; cat "$OUT/operator_ab.txt"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${4:-}" ]; then
  L=""; for x in $4; do L="$L trik-media-sensors-dsp_amd/$x"; done
  timeout -k 10 400 python scripts/blob_ab.py --frames 4096 --reps 5 $L > "$OUT/blob_ab.txt" 2>&1; rc=$?
  tail -6 "$OUT/blob_ab.txt"; [ $rc -eq 0 ] || exit $rc
fi
bash scripts/session_r04_tests.sh "$TAG" "${2:-}" "${5:-tests}"
