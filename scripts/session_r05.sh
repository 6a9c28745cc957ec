#!/bin/bash
# GPU box, round 5 (development): optional A/Bs, then optional tests and the
# driver's bench command; stops at the first failure.  Everything optional is
# passed in the environment:
#   KB="flags|libs;flags|libs"   scripts/kbench runs (libs relative to trik-media-sensors-dsp_amd/)
#   RANGE="libs"                 scripts/blob_ab.py --what range (autoDetectHsv)
#   BLOB="libs"                  scripts/blob_ab.py (multi-blob)
#   OP="libs"                    scripts/operator_ab.sh (scripts/bench_operator.py per library)
#   TESTS="pytest selection"     -m gpu tests
#   BENCH=1                      the driver's bench command (python bench.py --gpus 1 --steps 20 --warmup 5)
#   EXTRA="command"              one more command (its own timeout inside)
#   bash scripts/session_r05.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-t}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
P=trik-media-sensors-dsp_amd
if [ -n "${KB:-}" ]; then
  IFS=';' read -ra RUNS <<< "$KB"
  for R in "${RUNS[@]}"; do
    FLAGS="${R%%|*}"; LIBS="${R#*|}"; L=""
    for x in $LIBS; do L="$L $P/$x"; done
    echo "== kbench $FLAGS" >> "$OUT/kbench.txt"
    timeout -k 10 300 ./scripts/kbench $FLAGS $L >> "$OUT/kbench.txt" 2>&1; rc=$?
    [ $rc -eq 0 ] || { cat "$OUT/kbench.txt"; exit $rc; }
  done
  grep -v "^MISMATCH" "$OUT/kbench.txt" | sed "s#$P/##"
fi
if [ -n "${RANGE:-}" ]; then
  L=""; for x in $RANGE; do L="$L $P/$x"; done
  timeout -k 10 400 python scripts/blob_ab.py --what range --frames 4096 --reps 5 $L > "$OUT/range_ab.txt" 2>&1; rc=$?
  tail -12 "$OUT/range_ab.txt"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BLOB:-}" ]; then
  L=""; for x in $BLOB; do L="$L $P/$x"; done
  timeout -k 10 400 python scripts/blob_ab.py --frames 4096 --reps 5 $L > "$OUT/blob_ab.txt" 2>&1; rc=$?
  tail -12 "$OUT/blob_ab.txt"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${OP:-}" ]; then
  bash scripts/operator_ab.sh "$OUT/op" $OP > "$OUT/operator_ab.txt" 2>&1; rc=$?; cat "$OUT/operator_ab.txt"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "[s] tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${EXTRA:-}" ]; then
  bash -c "$EXTRA" > "$OUT/extra.txt" 2>&1; rc=$?; tail -20 "$OUT/extra.txt"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err"; rc=$?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])" "$OUT/bench_driver.json" || tail -5 "$OUT/bench_driver.err"
  exit $rc
fi
