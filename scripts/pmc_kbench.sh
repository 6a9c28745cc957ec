#!/bin/bash
# PMC passes (scripts/pmc_groups.txt minus FETCH/TCC) over kbench for each
# library given (development only; one counter group per rocprofv3 run).
# usage (GPU box): bash scripts/pmc_kbench.sh "kbench flags" lib1 [lib2 ...]
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/pmck"; mkdir -p "$OUT"
FLAGS="$1"; shift
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  N=$(echo "$L" | tr '/' '_'); mkdir -p "$OUT/$N"
  i=0
  for GROUP in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
               "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d "$OUT/$N/p$i" -o run \
      -- "$GRAFT_REPO_ROOT/scripts/kbench" $FLAGS "$GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$L" > "$OUT/$N/p$i.log" 2>&1
    rc=$?; echo "[pmc] $L group $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 "$GRAFT_REPO_ROOT/scripts/pmc_summary.py" "$OUT/$N" chroma_kernel 2516582400 > "$OUT/$N/summary.json" 2>&1
  python3 - "$OUT/$N/summary.json" "$L" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["counters_avg_per_launch"]
w = d["SQ_WAVE_CYCLES"]
print(sys.argv[2], "VALU %.1fM SALU %.1fM LDS %.1fM | wait_any %.2f wait_inst %.2f active %.2f | lds_conf %.2f | gui %.2fM"
      % (d["SQ_INSTS_VALU"]/1e6, d["SQ_INSTS_SALU"]/1e6, d["SQ_INSTS_LDS"]/1e6, d["SQ_WAIT_ANY"]/w,
         d["SQ_WAIT_INST_ANY"]/w, d["SQ_ACTIVE_INST_ANY"]/w, d["SQ_LDS_BANK_CONFLICT"]/max(1, d["SQ_LDS_IDX_ACTIVE"]),
         d["GRBM_GUI_ACTIVE"]/1e6))
PY
done
