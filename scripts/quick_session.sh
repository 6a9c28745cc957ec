#!/bin/bash
# GPU tests + bench + kernel-trace stats + PMC groups in one gpurun call; stops
# at the first fault / timeout.  usage: bash scripts/quick_session.sh TAG [--no-pmc]
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG="${1:-q}"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests_$TAG.log" 2>&1
rc=$?; echo "[q] tests rc=$rc"; tail -3 "$OUT/gpu_tests_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "[q] bench rc=$rc"; tail -1 "$OUT/bench_$TAG.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])" || tail -5 "$OUT/bench_$TAG.log"
[ $rc -eq 0 ] || exit $rc
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1 )
rc=$?; echo "[q] rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep -h "chroma_kernel\|stripe_kernel" "$OUT/prof_$TAG/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-60,120- || true
[ "${2:-}" = "--no-pmc" ] && exit 0
bash scripts/pmc_session.sh "pmc_$TAG"
