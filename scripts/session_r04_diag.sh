#!/bin/bash
# Round-4 diagnosis (GPU box): SALU/VALU/EXEC issue microbenchmarks, the
# driver's bench command twice, a kernel trace of that exact command (per-launch
# durations in order: the clock-ramp question), and the default 200-step bench.
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-r04a}"; mkdir -p "$OUT"
timeout -k 10 60 ./scripts/ubench/issue_mix > "$OUT/ubench_issue_mix.txt" 2>&1 || exit $?
timeout -k 10 60 ./scripts/ubench/exec_mix > "$OUT/ubench_exec_mix.txt" 2>&1 || exit $?
cat "$OUT/ubench_issue_mix.txt" "$OUT/ubench_exec_mix.txt"
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_$i.json" 2> "$OUT/bench_driver_$i.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/bench_driver_$i.json"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_driver" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/trace_driver.log" 2>&1 ) || exit $?
echo "[diag] trace ok"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_200.json" 2> "$OUT/bench_200.err" || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('200-step', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/bench_200.json"
