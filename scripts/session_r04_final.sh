#!/bin/bash
# GPU box, round 4 end: the GPU suite, smoke(), the driver's bench command for
# C3 and a C4 line, then rocprofv3 kernel stats and PMC of the driver command
# (scripts/session_r04_prof.sh).  Stops at the first failure.
#   bash scripts/session_r04_final.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-final}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
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
