# round-5 preview_rows2_kernel occupancy / memory-parallelism variants
FILE = "trik_hsv_operator.hip"
R2 = ("constexpr int kRowsQ = 1;  // units per lane and round (8 output pixels: 2 spill at 64 VGPRs)",
      "constexpr int kRowsQ = 2;  // units per lane and round (8 output pixels: 2 spill at 64 VGPRs)")
EU4 = ("""__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8)))
void preview_rows2_kernel(PreviewArgs a, PreviewRowsGeom g) {""",
       """__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
void preview_rows2_kernel(PreviewArgs a, PreviewRowsGeom g) {""")
GRID1 = ("const int64_t blocks = (total + 1024LL * kRowsQ - 1) / (1024LL * kRowsQ), slots = 2LL * device_cus();",
         "const int64_t blocks = (total + 1024LL * kRowsQ - 1) / (1024LL * kRowsQ), slots = 1LL * device_cus();")
VARIANTS = {
    "pv_base": [("constexpr int kRangeBlock = 256;", "constexpr int kRangeBlock = 256;")],
    "pv_q2": [R2, EU4],
    "pv_q2g1": [R2, EU4, GRID1],
    "pv_g1": [GRID1],
    "pv_q3g1": [(R2[0], R2[1].replace("kRowsQ = 2", "kRowsQ = 3")), EU4, GRID1],
}
