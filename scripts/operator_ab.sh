#!/bin/bash
# A/B of scripts/bench_operator.py over libtrik_hsv.so variants (development
# only; GPU box): each variant runs in its own process with a private copy of
# the host package.  usage: bash scripts/operator_ab.sh OUTDIR lib1 [lib2 ...]
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$1"; shift; mkdir -p "$OUT"
k=0
for L in "$@"; do
  k=$((k+1)); D=$(mktemp -d); mkdir -p "$D/trik_hsv"
  cp trik-media-sensors-dsp_amd/trik_hsv/*.py "$D/trik_hsv/"; cp "trik-media-sensors-dsp_amd/$L" "$D/trik_hsv/libtrik_hsv.so"
  TRIK_HSV_PKG_DIR="$D" timeout -k 10 300 python scripts/bench_operator.py --no-cpu > "$OUT/op_$k.json" 2> "$OUT/op_$k.err"; rc=$?
  rm -rf "$D"
  [ $rc -eq 0 ] || { tail -5 "$OUT/op_$k.err"; exit $rc; }
  python3 - "$L" "$OUT/op_$k.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
def g(k):
    v = d.get(k, {})
    return {kk: v[kk] for kk in v if kk in ("ms", "frac", "kernel_ms")} if isinstance(v, dict) else v
print(sys.argv[1], {k: g(k) for k in d if k in ("preview", "line_preview", "blob", "auto_range", "line")})
PY
done
