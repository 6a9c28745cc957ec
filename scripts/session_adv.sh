#!/bin/bash
# GPU box (development only): AUTO tests, the step gap with and without AUTO's
# probes, and the adversarial range-set table.
#   usage: bash scripts/session_adv.sh TAG [frames]
set -u
cd "$GRAFT_REPO_ROOT"; OUT="gpurun_out/$1"; mkdir -p "$OUT"; F="${2:-4096}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_auto.py tests/test_gpu_chroma.py tests/test_gpu_fused.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 3; }
tail -1 "$OUT/tests.log"
for h in chroma auto; do
  timeout -k 10 300 python bench.py --hot $h --no-extras --no-cpu-baseline > "$OUT/bench_$h.log" 2>&1 || { tail -20 "$OUT/bench_$h.log"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'gap_us', round(1000*(d['ms_per_step']-d['roofline']['kernel_ms']),2))" "$OUT/bench_$h.log" $h
done
timeout -k 10 900 python -u scripts/adversarial_ranges.py "$F" > "$OUT/adversarial.txt" 2>&1 || { tail -20 "$OUT/adversarial.txt"; exit 3; }
cat "$OUT/adversarial.txt"
