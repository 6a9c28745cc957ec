# development probe (GPU box): bench warmup/steps sensitivity
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/probe; mkdir -p $OUT
for ws in "3 20" "50 200" "200 500"; do
  set -- $ws
  timeout -k 10 120 python bench.py --no-cpu-baseline --warmup $1 --steps $2 > $OUT/bench_w$1_s$2.log 2>&1 || exit $?
  tail -1 $OUT/bench_w$1_s$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w=$1 s=$2', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 120 ./scripts/kbench -n 200 -r 3 trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so
