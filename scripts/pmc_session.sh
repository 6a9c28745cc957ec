#!/bin/bash
# PMC counter passes over a short bench run (one counter group per rocprofv3 run;
# no --sys-trace / --runtime-trace, per the pool rules).
set -u
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
TAG="${1:-pmc}"
shift || true
ARGS="${*:---steps 3 --warmup 1 --no-cpu-baseline --no-extras}"
mkdir -p "$OUT/$TAG"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $GROUP --output-format csv -d "$OUT/$TAG/p$i" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$OUT/$TAG/p$i.log" 2>&1
  rc=$?; echo "[pmc] group $i ($GROUP) rc=$rc" | tee -a "$OUT/$TAG/session.log"
  [ $rc -eq 0 ] || exit $rc
done < "$GRAFT_REPO_ROOT/scripts/pmc_groups.txt"
echo "[pmc] done" | tee -a "$OUT/$TAG/session.log"
