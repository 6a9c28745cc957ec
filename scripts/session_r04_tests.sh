#!/bin/bash
# GPU box: optional kbench A/B first ($2 = "flags|lib lib ..."), then the GPU
# test suite, then the driver's bench command; stops at the first failure.
#   bash scripts/session_r04_tests.sh TAG ["kbench flags|libs;flags|libs"] [pytest selection]
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-t}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
if [ -n "${2:-}" ]; then  # kbench runs: "flags|libs;flags|libs;..."
  IFS=';' read -ra RUNS <<< "$2"; k=0
  for R in "${RUNS[@]}"; do
    k=$((k+1)); FLAGS="${R%%|*}"; LIBS="${R#*|}"; L=""
    for x in $LIBS; do L="$L $GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$x"; done
    echo "== kbench $FLAGS" >> "$OUT/kbench.txt"
    timeout -k 10 300 ./scripts/kbench $FLAGS $L >> "$OUT/kbench.txt" 2>&1; rc=$?
    [ $rc -eq 0 ] || { cat "$OUT/kbench.txt"; exit $rc; }
  done
  grep -v "^MISMATCH" "$OUT/kbench.txt" | sed "s#$GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/##"
fi
SEL="${3:-tests}"
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "[s] tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err"; rc=$?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/bench_driver.json" || tail -5 "$OUT/bench_driver.err"
exit $rc
