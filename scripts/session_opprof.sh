#!/bin/bash
# GPU box: rocprofv3 kernel stats of the operator bench (SURVEY 8(f) kernels)
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/opprof"; mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_operator.py" --no-cpu > "$OUT/bench.log" 2>&1 ) || { tail -20 "$OUT/bench.log"; exit 3; }
cut -d, -f1-4 "$OUT/prof/run_kernel_stats.csv" | cut -c1-150 | head -30
