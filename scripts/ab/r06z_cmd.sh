set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/session_r06.sh r06z kbench "r6z_base drain2 tree" || exit 1
cp trik-media-sensors-dsp_amd/ab/drain2/libtrik_hsv.so trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_chroma.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_bench_call.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06z/tests_drain2.log 2>&1
echo "[r06z] drain2 tests rc=$?"; tail -2 gpurun_out/r06z/tests_drain2.log
