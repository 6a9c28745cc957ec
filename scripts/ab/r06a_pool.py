# round-6 A/B: the fused step's tail pool (kPoolPermille of the batch's units
# taken one by one from a device counter by workgroups done with their own
# share) against the round-5 kernel (REV=HEAD: even static shares only)
FILE = "trik_hsv_chroma.hip"
_T = __import__("runpy").run_path(__file__.replace("r06a_pool.py", "trace.py"))["VARIANTS"]["trace"]
P = "constexpr uint32_t kPoolPermille = 100;"
VARIANTS = {
    "r5base": ["REV=c0cbf67"],
    "pool0": [(P, "constexpr uint32_t kPoolPermille = 0;")],
    "pool50": [(P, "constexpr uint32_t kPoolPermille = 50;")],
    "pool100": [(P, P)],
    "pool200": [(P, "constexpr uint32_t kPoolPermille = 200;")],
    "tr_pool0": [(P, "constexpr uint32_t kPoolPermille = 0;")] + _T,
    "tr_pool100": list(_T),
}
