#!/bin/bash
# One GPU session on the box: GPU tests, smoke, bench, rocprofv3 kernel-trace stats.
# Stops at the first step that times out / aborts / faults (exit >= 2 from pytest,
# or any non-zero from the others).
set -u
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-r01}"
echo "[session] $(date) tag=$TAG" | tee "$OUT/session.log"
rocm-smi --showproductname --showmeminfo vram > "$OUT/rocm_smi.txt" 2>&1 || true

timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[session] gpu tests rc=$rc" | tee -a "$OUT/session.log"
tail -5 "$OUT/gpu_tests.log" | tee -a "$OUT/session.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "[session] smoke rc=$rc" | tee -a "$OUT/session.log"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "[session] bench rc=$rc" | tee -a "$OUT/session.log"; tail -1 "$OUT/bench.log" | tee -a "$OUT/session.log"; [ $rc -eq 0 ] || exit $rc

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "[session] rocprof rc=$rc" | tee -a "$OUT/session.log"; [ $rc -eq 0 ] || exit $rc
find "$OUT/prof_$TAG" -name "*stats*" | tee -a "$OUT/session.log"
echo "[session] done $(date)" | tee -a "$OUT/session.log"
