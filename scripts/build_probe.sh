#!/bin/bash
# GPU box (development only): the builder kernels' times for library variants
# (rocprofv3 kernel stats over scripts/cold_probe.py on a copy of the package).
#   usage: bash scripts/build_probe.sh lib...   (dirs under trik-media-sensors-dsp_amd/ab, or "prod")
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bp
for x in "$@"; do
  P=/tmp/bp_pkg_$x; rm -rf $P; mkdir -p $P; cp -r trik-media-sensors-dsp_amd/trik_hsv $P/
  [ "$x" = prod ] || cp trik-media-sensors-dsp_amd/ab/$x/libtrik_hsv.so $P/trik_hsv/libtrik_hsv.so
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/bp/$x" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/cold_probe.py" $P > "$GRAFT_REPO_ROOT/gpurun_out/bp/$x.log" 2>&1 ) \
    || { tail -20 "gpurun_out/bp/$x.log"; exit 3; }
  echo "== $x"; grep -E "chroma_(summary|block)|compile_tables" "gpurun_out/bp/$x/run_kernel_stats.csv" | cut -d, -f1,2,4 | cut -c1-140
done
