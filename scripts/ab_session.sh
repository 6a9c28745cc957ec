#!/bin/bash
# A/B of kernel library variants: bench (kernel ms) + PMC for each.
# usage: bash scripts/ab_session.sh TAG lib1 [lib2 ...]   (paths relative to repo)
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG="$1"; shift; mkdir -p "$OUT/ab_$TAG"
for LIB in "$@"; do
  N=$(basename $(dirname "$LIB"))
  TRIK_HSV_LIB="$GRAFT_REPO_ROOT/$LIB" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > "$OUT/ab_$TAG/bench_$N.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "[ab] $N bench rc=$rc"; tail -3 "$OUT/ab_$TAG/bench_$N.log"; exit $rc; }
  tail -1 "$OUT/ab_$TAG/bench_$N.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[ab] $N kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
  if [ "${AB_PMC:-0}" = 1 ]; then
    TRIK_HSV_LIB="$GRAFT_REPO_ROOT/$LIB" bash scripts/pmc_session.sh "ab_$TAG/pmc_$N" || exit $?
  fi
done
