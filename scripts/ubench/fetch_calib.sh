#!/bin/bash
# GPU box: timing + two PMC passes (FETCH_SIZE; TCC requests/hits/misses) over
# scripts/ubench/fetch_calib.  usage: bash scripts/ubench/fetch_calib.sh OUTDIR
set -u
OUT="$(realpath -m "$1")"; mkdir -p "$OUT"
BIN="$GRAFT_REPO_ROOT/scripts/ubench/fetch_calib"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 "$BIN" > "$OUT/fetch_calib_time.txt" 2>&1 || exit $?
cat "$OUT/fetch_calib_time.txt"
i=0
for GROUP in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d "$OUT/fc$i" -o run -- "$BIN" \
    > "$OUT/fc$i.log" 2>&1 || exit $?
  echo "[fetch_calib] pass $i ($GROUP) ok"
done
