#!/bin/bash
# GPU box: blob/preview A/B (scripts/blob_ab.py, scripts/bench_operator.py)
# then the given session (scripts/session_r04_tests.sh args).
#   bash scripts/session_r04_blob.sh TAG "blob libs" [session_r04_tests args...]
set -u
cd "$GRAFT_REPO_ROOT"; TAG="$1"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
L=""; for x in $2; do L="$L trik-media-sensors-dsp_amd/$x"; done
timeout -k 10 300 python scripts/blob_ab.py --frames 4096 --reps 5 $L > "$OUT/blob_ab.txt" 2>&1; rc=$?
cat "$OUT/blob_ab.txt" | tail -8; [ $rc -eq 0 ] || exit $rc
shift 2
[ $# -gt 0 ] && exec_args=("$@") && bash scripts/session_r04_tests.sh "$TAG" "${exec_args[@]}"
