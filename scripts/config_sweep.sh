#!/bin/bash
# Hot-kernel time across the BASELINE configs (uniform and scene frames), one line each.
# usage: bash scripts/config_sweep.sh OUTFILE
set -u
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-sweep.txt}"; : > "$OUT"
run() {  # label, bench args
  local L="$1"; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/sweep_b.log 2>&1 || { echo "$L FAILED"; tail -3 gpurun_out/sweep_b.log; exit 1; }
  tail -1 gpurun_out/sweep_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%-34s %-22s kernel_ms %.4f  Mpix/s %.0f  frac %.3f' % ('$L', r['kernel'], r['kernel_ms'], d['value'], r['frac']))" | tee -a "$OUT"
}
run "C3 4096x640x480 T=4 uniform"
run "C3 4096x640x480 T=4 scene" --kind 1
run "C3 shape T=2 uniform" --targets 2
run "C3 shape T=1 uniform" --targets 1
run "C4 1024x1280x720 T=2 uniform" --frames 1024 --width 1280 --height 720 --targets 2
run "C4 1024x1280x720 T=2 scene" --frames 1024 --width 1280 --height 720 --targets 2 --kind 1
run "C3 4096x640x480 T=4 stripe kernel" --hot stripe
