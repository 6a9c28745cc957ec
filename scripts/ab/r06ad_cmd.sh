set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/session_r06.sh r06ad blob "r6ad_base bdrain2 tree" blob || exit 1
cp trik-media-sensors-dsp_amd/ab/bdrain2/libtrik_hsv.so trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_blob.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06ad/tests_bdrain2.log 2>&1
echo "[r06ad] bdrain2 tests rc=$?"; tail -2 gpurun_out/r06ad/tests_bdrain2.log
