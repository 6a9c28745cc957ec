set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/session_r06.sh r06u blob "r6u_base hsv3 hsv3_kf tree" range || exit 1
cp trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so /tmp/tree.so
for v in hsv3 hsv3_kf; do
  cp trik-media-sensors-dsp_amd/ab/$v/libtrik_hsv.so trik-media-sensors-dsp_amd/trik_hsv/libtrik_hsv.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_operator.py tests/test_gpu_line.py tests/test_gpu_wline.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r06u/tests_$v.log 2>&1
  echo "[r06u] $v tests rc=$?"; tail -2 gpurun_out/r06u/tests_$v.log
done
