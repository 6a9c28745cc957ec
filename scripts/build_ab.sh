#!/bin/bash
# Builds chroma-kernel variants for timing attribution (development only):
#   bash scripts/build_ab.sh NAME "-DFLAG ..." [NAME "-DFLAG" ...]
# -> trik-media-sensors-dsp_amd/ab/NAME/libtrik_hsv.so (the other objects from build/)
set -eu
cd "$(dirname "$0")/../trik-media-sensors-dsp_amd"
make -s -C csrc >/dev/null
while [ $# -ge 2 ]; do
  N="$1"; D="$2"; shift 2; mkdir -p "ab/$N"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $D \
      -c -o "ab/$N/chroma.o" csrc/trik_hsv_chroma.hip
  objs=$(ls build/*.o | grep -v chroma)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "ab/$N/libtrik_hsv.so" "ab/$N/chroma.o" $objs
  echo "built ab/$N"
done
