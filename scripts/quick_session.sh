#!/bin/bash
# tests + bench + PMC groups (one call); stops on the first fault/timeout
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out"; TAG="${1:-q}"; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[q] tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc=$?; echo "[q] bench rc=$rc"; tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value',d['value'],'kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])" || tail -5 "$OUT/bench.log"
[ $rc -eq 0 ] || exit $rc
bash scripts/pmc_session.sh "pmc_$TAG"
