#!/bin/bash
# GPU box: the driver's bench command (C3), a C4 line and the operator bench,
# nothing else on the GPU before them (development; a second box's numbers).
#   bash scripts/session_r06_bench.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-bench}"; mkdir -p "$OUT"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit $?
timeout -k 10 300 python bench.py --gpus 1 --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit $?
timeout -k 10 400 python scripts/bench_operator.py --frames 4096 --no-cpu > "$OUT/operator_bench.json" 2> "$OUT/operator_bench.err" || exit $?
python3 -c "
import json
for f in ('bench_driver', 'bench_c4'):
    d = json.load(open('$OUT/' + f + '.json')); r = d['roofline']
    print(f, d['ms_per_step'], r['kernel_ms'], r['frac'], r['traffic'])
d = json.load(open('$OUT/operator_bench.json'))
print({k: v.get('ms') for k, v in d.items() if isinstance(v, dict)})"
