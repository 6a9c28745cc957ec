#!/bin/bash
# Builds libtrik_hsv.so variants whose chroma kernel source comes from a git
# revision or a file (development only):
#   bash scripts/build_ab_rev.sh NAME REV|FILE ["-DFLAG ..."] [NAME REV|FILE [FLAGS] ...]
# -> trik-media-sensors-dsp_amd/ab/NAME/libtrik_hsv.so (the other objects from build/)
set -eu
cd "$(dirname "$0")/../trik-media-sensors-dsp_amd"
make -s -C csrc >/dev/null
while [ $# -ge 2 ]; do
  N="$1"; R="$2"; shift 2; D=""
  if [ $# -ge 1 ] && [[ "$1" == -* ]]; then D="$1"; shift; fi
  mkdir -p "ab/$N"
  if [ -f "$R" ]; then cp "$R" "ab/$N/chroma.hip"; else git show "$R:trik-media-sensors-dsp_amd/csrc/trik_hsv_chroma.hip" > "ab/$N/chroma.hip"; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Icsrc $D \
      -c -o "ab/$N/chroma.o" "ab/$N/chroma.hip"
  objs=$(ls build/*.o | grep -v chroma)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "ab/$N/libtrik_hsv.so" "ab/$N/chroma.o" $objs
  echo "built ab/$N"
done
