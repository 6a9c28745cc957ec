#!/bin/bash
# GPU box, round 4: the evidence for the bench line -- rocprofv3 kernel stats
# of the driver's exact command, then the PMC passes (one counter group per
# run, scripts/pmc_groups.txt) and their summary for chroma_kernel.
#   bash scripts/session_r04_prof.sh TAG [nopmc]
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-prof}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/stats_bench.json" 2> "$OUT/stats_bench.err" ) || exit $?
echo "[prof] kernel stats ok"
python3 scripts/trace_timed.py "$OUT/stats/run_kernel_trace.csv" chroma_kernel 20 "$OUT/timed_launches.txt" > /dev/null && sed -n 1,3p "$OUT/timed_launches.txt"
[ "${2:-}" = nopmc ] && exit 0
bash scripts/pmc_session.sh "$TAG/pmc" || exit $?
python3 scripts/pmc_summary.py "$OUT/pmc" chroma_kernel 2516582400 "$OUT/pmc_summary.json" || exit $?
