#!/bin/bash
# GPU box (development only): the chroma-run builder's tests, the bench's
# cold-batch figures and the builder kernels' times.
#   usage: bash scripts/session_build.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$1"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_chroma.py tests/test_gpu_blob.py tests/test_gpu_fused.py tests/test_gpu_auto.py} \
  tests/test_gpu_streams.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 \
  || { tail -30 "$OUT/tests.log"; exit 3; }
tail -1 "$OUT/tests.log"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --scene-launches 0 > "$OUT/bench_$i.log" 2>&1 || { tail -20 "$OUT/bench_$i.log"; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('cold', d['cold_batch'])" "$OUT/bench_$i.log"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --scene-launches 0 > "$OUT/prof.log" 2>&1 ) || { tail -20 "$OUT/prof.log"; exit 3; }
grep -E "chroma_(summary|block)" "$OUT/prof/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-160
