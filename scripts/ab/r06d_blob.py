# round-6 A/B, multi-blob clusterer: round 5's one wave per frame (REV) against
# the two-wave row pipeline (labeler + bookkeeper) in the work tree
FILE = "trik_hsv_blob.hip"
VARIANTS = {
    "blob_r5": ["REV=c0cbf67"],
}
