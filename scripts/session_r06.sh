#!/bin/bash
# GPU box, round 6 (development sessions; each step stops the call at its
# first failure):
#   bash scripts/session_r06.sh TAG tests "PYTEST ARGS"   -- GPU tests
#   bash scripts/session_r06.sh TAG kbench "VARIANTS"     -- kbench C3/C4 full steps back to back
#   bash scripts/session_r06.sh TAG overlap [sum|auto] [nocomm] -- scripts/overlap_probe.py under rocprofv3
#   bash scripts/session_r06.sh TAG blob "LIBS"           -- scripts/blob_ab.py (multi-blob batch A/B)
set -u
cd "$GRAFT_REPO_ROOT"; TAG="${1:-r06}"; OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
case "${2:-tests}" in
tests)
  timeout -k 10 900 python -u -m pytest ${3:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "[r06] tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; exit $rc ;;
kbench)
  libs=""; for v in ${3}; do if [ "$v" = tree ]; then libs="$libs trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so"; else libs="$libs trik-media-sensors-dsp_amd/ab/$v/libtrik_hsv.so"; fi; done
  echo "== kbench -s -b -r 3 -n 30 (C3)" > "$OUT/kbench.txt"
  timeout -k 10 400 scripts/kbench -s -b -r 3 -n 30 $libs >> "$OUT/kbench.txt" 2>&1 || { echo "kbench c3 failed"; tail -5 "$OUT/kbench.txt"; exit 1; }
  echo "== kbench -s -b -r 3 -n 30 -f 1024 -w 1280 -h 720 -t 2 (C4)" >> "$OUT/kbench.txt"
  timeout -k 10 400 scripts/kbench -s -b -r 3 -n 30 -f 1024 -w 1280 -h 720 -t 2 $libs >> "$OUT/kbench.txt" 2>&1 || { echo "kbench c4 failed"; exit 1; }
  echo "[r06] kbench ok"; grep -E "back to back|median|MISMATCH|trace:" "$OUT/kbench.txt" | sed 's#trik-media-sensors-dsp_amd/##' ;;
overlap)
  for m in plain reserved; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ov_$m" -o run \
        -- python3 "$GRAFT_REPO_ROOT/scripts/overlap_probe.py" --mode $m --steps 30 --standin ${3:-sum} > "$OUT/ov_$m.json" 2> "$OUT/ov_$m.err" ) || { echo "overlap $m failed"; tail -5 "$OUT/ov_$m.err"; exit 1; }
    cat "$OUT/ov_$m.json"
    f=$(find "$OUT/ov_$m" -name "*kernel_trace.csv" | head -1)
    python3 scripts/overlap_trace.py "$f" "$OUT/ov_${m}_trace.txt" | head -3
  done
  timeout -k 10 300 python3 scripts/overlap_probe.py --mode all --steps 100 --standin ${3:-sum} > "$OUT/ov_timing.json" 2> "$OUT/ov_timing.err"
  echo "timing rc=$?"; cat "$OUT/ov_timing.json"
  [ "${4:-}" = nocomm ] && exit 0
  # bench.py's own collective path on one GPU (a one-rank library comm): does RCCL launch a kernel?
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ov_comm" -o run \
      -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-extras --no-cpu-baseline --comm-self > "$OUT/ov_comm.json" 2> "$OUT/ov_comm.err" ) || { echo "comm-self trace failed"; exit 1; }
  f=$(find "$OUT/ov_comm" -name "*kernel_trace.csv" | head -1)
  python3 -c "
import csv, collections
rows = list(csv.DictReader(open('$f')))
c = collections.Counter(r['Kernel_Name'][:80] for r in rows)
for k, v in c.most_common(12): print(v, k)"
  cat "$OUT/ov_timing.json" ;;
blob)
  libs=""; for v in ${3}; do if [ "$v" = tree ]; then libs="$libs trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so"; else libs="$libs trik-media-sensors-dsp_amd/ab/$v/libtrik_hsv.so"; fi; done
  timeout -k 10 600 python3 scripts/blob_ab.py --what ${4:-blob} --reps 5 $libs > "$OUT/blob_ab.txt" 2> "$OUT/blob_ab.err" || { echo "blob_ab failed"; tail -5 "$OUT/blob_ab.err"; exit 1; }
  cat "$OUT/blob_ab.txt" ;;
esac
