#!/bin/bash
# GPU box: PMC passes over autoDetectHsv on 4096 VGA scene frames (in-tree
# library), one counter group per rocprofv3 run (development).
#   bash scripts/range_pmc.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-rpmc}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for GROUP in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_EXP"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/range_time.py" --only scene > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[rpmc] group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "auto_range_vec_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    # one row per (dispatch, counter) after summing over dimensions is what rocprofv3 writes
    print(k, len(v), sum(v) / len(v))
PY
