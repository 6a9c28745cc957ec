set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/s1; mkdir -p $OUT
timeout -k 10 400 python scripts/blob_ab.py trik-media-sensors-dsp_amd/ab/base/libtrik_hsv.so trik-media-sensors-dsp_amd/ab/noreplay/libtrik_hsv.so trik-media-sensors-dsp_amd/ab/noatom/libtrik_hsv.so trik-media-sensors-dsp_amd/ab/noccl/libtrik_hsv.so > $OUT/blob_ab.txt 2>&1 || { cat $OUT/blob_ab.txt; exit 1; }
cat $OUT/blob_ab.txt
timeout -k 10 300 python scripts/bench_operator.py --no-cpu > $OUT/operator.json 2>&1 || { tail -5 $OUT/operator.json; exit 1; }
tail -c 3000 $OUT/operator.json
