#!/bin/bash
# GPU box: the given test files, then the C3 and C4 bench lines and the C4
# kernel-trace stats.  usage: bash scripts/session_new_tests.sh TAG test_file...
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG="$1"; shift; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/tests_$TAG.log" 2>&1
rc=$?; echo "[s] tests rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/tests_$TAG.log" | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench_c3_$TAG.log" 2>&1 || exit $?
tail -1 "$OUT/bench_c3_$TAG.log"
timeout -k 10 300 python bench.py --workload c4 --no-cpu-baseline > "$OUT/bench_c4_$TAG.log" 2>&1 || exit $?
tail -1 "$OUT/bench_c4_$TAG.log"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4_$TAG" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --no-cpu-baseline > "$OUT/prof_c4_$TAG.log" 2>&1 ) || exit $?
grep -h "chroma_kernel" "$OUT/prof_c4_$TAG/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-60,120-
