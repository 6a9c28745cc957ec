"""Helpers shared by the GPU parity tests (test code, not product)."""
import numpy as np

LAYOUT_YUYV, LAYOUT_OV7670 = 0, 1

T0 = (0, 30, 50, 100, 30, 100)
T1 = (90, 150, 40, 100, 20, 100)
T2 = (200, 260, 40, 100, 20, 100)
T3 = (330, 20, 30, 100, 30, 100)  # hue wrap
BENCH_RANGES = [T0, T1, T2, T3]


def exhaustive_yuyv_frame():
    """An 8192x2048 YUYV frame holding every (Y,U,V) triple exactly once.

    Pair p (row-major, 4096 pairs per row): U = p & 255, V = (p >> 8) & 255,
    Y0 = 2k, Y1 = 2k + 1 with k = p >> 16.
    """
    p = np.arange(1 << 23, dtype=np.uint32)
    u = p & 255
    v = (p >> 8) & 255
    k = p >> 16
    words = (2 * k) | (u << 8) | ((2 * k + 1) << 16) | (v << 24)
    return words.astype("<u4").view(np.uint8), 8192, 2048, 16384


def sums_from_mask(mask, n_ranges):
    """[H,W] bit masks -> [T,3] int64 {N, sumX, sumY}."""
    h, w = mask.shape
    xs = np.arange(w, dtype=np.int64)[None, :]
    ys = np.arange(h, dtype=np.int64)[:, None]
    out = np.zeros((n_ranges, 3), np.int64)
    for t in range(n_ranges):
        d = ((mask >> t) & 1).astype(np.int64)
        out[t] = [d.sum(), (d * xs).sum(), (d * ys).sum()]
    return out
