# round-6 A/B, autoDetectHsv (auto_range_vec_kernel): batch slots past the
# zone for the whole wave skip their HSV (work tree) against round 6's start
FILE = "trik_hsv_operator.hip"
VARIANTS = {
    "range_r5": ["REV=c0cbf67"],
}
