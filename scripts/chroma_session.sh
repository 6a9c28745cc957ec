#!/bin/bash
# Chroma-run kernel: its GPU parity tests, then bench (auto, stripe) and a
# kernel-trace stats run.  usage: bash scripts/chroma_session.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG="${1:-c}"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_chroma.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/chroma_tests_$TAG.log" 2>&1
rc=$?; echo "[c] chroma tests rc=$rc"; tail -15 "$OUT/chroma_tests_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for hot in chroma stripe; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --hot $hot > "$OUT/bench_${TAG}_$hot.log" 2>&1
  rc=$?; echo "[c] bench $hot rc=$rc"; tail -1 "$OUT/bench_${TAG}_$hot.log" | cut -c1-100; tail -1 "$OUT/bench_${TAG}_$hot.log" | grep -o '"roofline".*' | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --hot chroma > "$OUT/prof_$TAG.log" 2>&1 )
rc=$?; echo "[c] rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
cut -d, -f1-8 "$OUT/prof_$TAG/run_kernel_stats.csv" | head -12
