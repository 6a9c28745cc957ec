# round-6 A/B, autoDetectHsv: the pixel pair's H, S, V handed to the counting
# as three values (no packed key to pack and unpack: -5 VALU per pixel pair)
#  split   the work tree;  r6w_head: the committed form (REV=HEAD)
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "r6w_head": ["REV=HEAD"],
    "split": [("kVecBatch = 4;", "kVecBatch = 4;")],
}
