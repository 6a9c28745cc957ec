// Development check (not a test): the interval form of the sv table in
// compile_tables (csrc/trik_hsv_tables.cpp) against the per-(mx, mn) loop it
// replaced, on 20,000 random range sets.  build + run:
//   hipcc -O2 -std=c++17 -Itrik-media-sensors-dsp_amd/csrc -Iinclude -x hip --offload-arch=gfx950 \
//     scripts/debug/sv_interval_check.cpp trik-media-sensors-dsp_amd/csrc/trik_hsv_tables.cpp -o /tmp/svc && /tmp/svc
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "trik_hsv_internal.h"
using namespace trik_hsv;
// the previous per-(mx, mn) loop, as the reference for the interval form
static void old_sv(const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, const uint16_t* lut255, uint8_t* sv) {
  memset(sv, 0, 65536);
  for (int t = 0; t < n; ++t) {
    PackedRange p = pack_range(ranges[t]);
    uint32_t fs = (p.from >> 8) & 0xFF, ts = (p.to >> 8) & 0xFF, fv = (p.from >> 16) & 0xFF, tv = (p.to >> 16) & 0xFF;
    for (uint32_t mx = 0; mx < 256; ++mx) {
      if (mx < fv || mx > tv) continue;
      for (uint32_t mn = 0; mn <= mx; ++mn) {
        uint32_t s = (lut255[mx] * (mx - mn)) >> 8;
        if (!(s < fs || s > ts)) sv[mx * 256 + mn] |= (uint8_t)(1u << t);
      }
    }
  }
}
int main() {
  static RangeTables t; static uint8_t ref[65536];
  srand(7); long bad = 0;
  for (int it = 0; it < 20000; ++it) {
    TRIK_VIDTRANSCODE_CV_InArgsAlg r[4] = {};
    for (int i = 0; i < 4; ++i) {
      r[i].detectHueFrom = rand() % 400; r[i].detectHueTo = rand() % 400;
      r[i].detectSatFrom = rand() % 120 - 10; r[i].detectSatTo = rand() % 120 - 10;
      r[i].detectValFrom = rand() % 120 - 10; r[i].detectValTo = rand() % 120 - 10;
      if (it % 7 == 0) { r[i].detectSatFrom = 0; r[i].detectSatTo = 100; }
      if (it % 11 == 0) { r[i].detectValFrom = rand() % 3; r[i].detectValTo = rand()%3 ? 100 : 0; }
    }
    compile_tables(r, 4, &t);
    old_sv(r, 4, t.lut255, ref);
    if (memcmp(ref, t.sv, 65536)) ++bad;
  }
  printf("bad %ld of 20000\n", bad);
  return bad != 0;
}
