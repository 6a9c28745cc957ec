#!/bin/bash
# GPU box (development only): kbench A/B of library variants on C3 uniform,
# C3 scene and C4, then the given GPU test files.
#   bash scripts/ab_session.sh TAG "lib1 lib2 ..." [test files...]
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/ab_$1"; mkdir -p "$OUT"; LIBS="$2"; shift 2
L=""; for x in $LIBS; do L="$L $GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$x"; done
K="$GRAFT_REPO_ROOT/scripts/kbench"
timeout -k 10 200 $K -n 50 -r 3 $L > "$OUT/c3.txt" 2>&1 || { cat "$OUT/c3.txt"; exit 3; }
cat "$OUT/c3.txt"
timeout -k 10 200 $K -n 50 -r 2 -k 1 $L > "$OUT/c3_scene.txt" 2>&1 || { cat "$OUT/c3_scene.txt"; exit 3; }
cat "$OUT/c3_scene.txt"
timeout -k 10 200 $K -n 50 -r 2 -f 1024 -w 1280 -h 720 -t 2 $L > "$OUT/c4.txt" 2>&1 || { cat "$OUT/c4.txt"; exit 3; }
cat "$OUT/c4.txt"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; grep -E "passed|failed|FAIL|ERROR" "$OUT/tests.log" | tail -12; exit $rc
fi
