#!/bin/bash
# GPU box, round 6 evidence (stops at its first failure):
#   bash scripts/session_r06_final.sh TAG main -- the GPU suite, smoke(), the
#     driver's bench command (C3) and a C4 line, rocprofv3 kernel stats of the
#     driver command with its timed launches, the PMC passes and their summary
#   bash scripts/session_r06_final.sh TAG ops  -- scripts/bench_operator.py and
#     its rocprofv3 kernel stats
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-final}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ "${2:-main}" = main ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "[final] tests rc=$rc"; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "[final] smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit $?
  timeout -k 10 300 python bench.py --gpus 1 --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit $?
  python3 -c "
import json
for f in ('bench_driver', 'bench_c4'):
    d = json.load(open('$OUT/' + f + '.json')); r = d['roofline']
    print(f, d['ms_per_step'], r['kernel_ms'], r['frac'], r['traffic'])"
  bash scripts/session_r04_prof.sh "$TAG"
else
  timeout -k 10 400 python scripts/bench_operator.py --frames 4096 > "$OUT/operator_bench.json" 2> "$OUT/operator_bench.err"
  rc=$?; echo "[final] operator bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/opstats" -o run \
      -- python3 "$GRAFT_REPO_ROOT/scripts/bench_operator.py" --frames 4096 --no-cpu > "$OUT/opstats_bench.json" 2> "$OUT/opstats_bench.err" ) || exit $?
  echo "[final] operator kernel stats ok"
fi
