#!/bin/bash
# A/B of chroma-kernel library variants (kernel ms at T=4 and T=1).
# usage: bash scripts/ab_chroma.sh lib1 [lib2 ...]  (paths relative to trik-media-sensors-dsp_amd/)
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/ab; mkdir -p $OUT
for L in "$@"; do
  for T in 4 1; do
    TRIK_HSV_LIB="$GRAFT_REPO_ROOT/trik-media-sensors-dsp_amd/$L" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --targets $T --hot chroma > $OUT/b.log 2>&1 || { tail -3 $OUT/b.log; exit 1; }
    tail -1 $OUT/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L T=$T', d['roofline']['kernel_ms'], d['roofline']['frac'])"
  done
done
