#!/bin/bash
# GPU box: PMC passes over the multi-blob batch (scripts/blob_time.py, 4096
# ov7670 VGA scene frames, in-tree library), one counter group per rocprofv3
# run; per-kernel averages of blob_chroma_meta_kernel and blob_ccl_kernel.
#   bash scripts/blob_pmc.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-bpmc}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for GROUP in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d "$OUT/p$i" -o run \
    -- python3 "$GRAFT_REPO_ROOT/scripts/blob_time.py" 4096 1 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "[bpmc] group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for k in ("blob_chroma_meta_kernel", "blob_ccl_kernel"):
            if k in r["Kernel_Name"]:
                acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(k, c, len(v), sum(v) / len(v))
PY
