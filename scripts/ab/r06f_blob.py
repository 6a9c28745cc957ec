# round-6 A/B, multi-blob clusterer (one wave per frame):
#  blob_r5   round 5 (REV)
#  acc       statistics runs carried across rows (a lane adds once per blob,
#            not once per row) + the row batch as packed bits (work tree)
# (round 6 first tried two waves per frame a row apart -- a labeler and a
# bookkeeper, one barrier per row: correct, but slower in r06d, 1.057 ->
# 1.209 ms uniform, 0.797 -> 0.878 ms scenes; not kept)
FILE = "trik_hsv_blob.hip"
VARIANTS = {
    "blob_r5": ["REV=c0cbf67"],
    "acc": [("  int next = 1;  // next new label (wave-uniform)\n", "  int next = 1;  // next new label (wave-uniform)\n")],
}
