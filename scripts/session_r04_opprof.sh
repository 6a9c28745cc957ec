#!/bin/bash
# GPU box, round 4: the operator kernels (scripts/bench_operator.py) under
# rocprofv3 -- kernel stats, then PMC passes (one counter group per run).
#   bash scripts/session_r04_opprof.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-opprof}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
  -- python3 "$GRAFT_REPO_ROOT/scripts/bench_operator.py" --frames 4096 --iters 5 --no-cpu > "$OUT/stats.json" 2> "$OUT/stats.err" || exit $?
echo "[opprof] stats ok"
i=0
for GROUP in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/bench_operator.py" --frames 4096 --iters 2 --no-cpu > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[opprof] group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
