#!/bin/bash
# GPU box: the given GPU test files, the C3 and C4 bench lines, and the
# rocprofv3 kernel stats of the C3 bench command.
#   bash scripts/session_round.sh TAG [test files...]   (no files: tests skipped)
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$1"; TAG="$1"; shift; mkdir -p "$OUT"
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
  rc=$?; echo "[s] tests rc=$rc"; grep -E "passed|failed|FAIL|ERROR" "$OUT/tests.log" | tail -12
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > "$OUT/bench_c3.log" 2>&1 || { tail -20 "$OUT/bench_c3.log"; exit 3; }
tail -1 "$OUT/bench_c3.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_c3_driver.log" 2>&1 || { tail -20 "$OUT/bench_c3_driver.log"; exit 3; }
tail -1 "$OUT/bench_c3_driver.log"
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > "$OUT/bench_c4.log" 2>&1 || { tail -20 "$OUT/bench_c4.log"; exit 3; }
tail -1 "$OUT/bench_c4.log"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_c3.log" 2>&1 ) || { tail -20 "$OUT/prof_c3.log"; exit 3; }
cut -d, -f1-4 "$OUT/prof_c3/run_kernel_stats.csv" | cut -c1-150 | head -12
