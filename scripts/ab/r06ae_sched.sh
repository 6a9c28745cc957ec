#!/bin/bash
# round-6 A/B, hot kernel: the same source under LLVM's other AMDGPU machine
# schedulers (-mllvm -amdgpu-sched-strategy=...), linked like ab_variants.py's
# variants into trik-media-sensors-dsp_amd/ab/NAME/libtrik_hsv.so
set -eu
cd "$(dirname "$0")/../../trik-media-sensors-dsp_amd"
make -s -C csrc >/dev/null
for st in max-ilp max-memory-clause iterative-ilp; do
  mkdir -p ab/s_$st
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Icsrc \
      -mllvm -amdgpu-sched-strategy=$st -c -o ab/s_$st/var.o csrc/trik_hsv_chroma.hip
  objs=$(ls build/*.o | grep -v "/trik_hsv_chroma.hip.o")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ab/s_$st/libtrik_hsv.so ab/s_$st/var.o $objs -ldl -lpthread
  echo "built ab/s_$st"
done
