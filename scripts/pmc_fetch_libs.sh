#!/bin/bash
# FETCH_SIZE per chroma_kernel launch for each library given (development
# only): one rocprofv3 --pmc FETCH_SIZE pass over a short kbench run each.
# usage (GPU box): bash scripts/pmc_fetch_libs.sh OUTDIR "kbench flags" lib1 [lib2 ...]
set -u
OUT="$(realpath -m "$1")"; FLAGS="$2"; shift 2; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  N=$(echo "$L" | tr '/' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/$N" -o run \
    -- "$GRAFT_REPO_ROOT/scripts/kbench" $FLAGS "$GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$L" > "$OUT/$N.log" 2>&1 || exit $?
  python3 - "$OUT/$N/run_counter_collection.csv" "$L" <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "chroma_kernel" in r["Kernel_Name"]]
v = v[3:] if len(v) > 6 else v
print(sys.argv[2], "chroma_kernel FETCH_SIZE x2 / algorithmic: %.4f over %d launches" % (sum(v) / len(v) * 2048 / 2516582400, len(v)))
PY
done
