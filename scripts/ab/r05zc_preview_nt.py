# round-5 A/B: the 2:1 preview's stores nontemporal (630 MB written per 4096
# VGA frames; back-to-back batches slow from 0.38 to 0.48 ms as the writes
# pile up behind the L2/MALL)
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "pv_base": [("constexpr int kRangeBlock = 256;", "constexpr int kRangeBlock = 256;")],
    "pv_ntst": [("""          *reinterpret_cast<uint2*>(dst + 8 * h) = o;""",
                 """          typedef unsigned int v2u __attribute__((ext_vector_type(2)));
          v2u ov;
          ov.x = o.x;
          ov.y = o.y;
          __builtin_nontemporal_store(ov, reinterpret_cast<v2u*>(dst + 8 * h));""")],
}
