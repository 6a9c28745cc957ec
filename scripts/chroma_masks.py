"""The exhaustive per-chroma mask profiles (development analysis, CPU only):
mask[c, Y] for c = U | V << 8 and Y = 0..255 under the bench ranges, from the
oracle (oracle/trik_oracle.c: WSEQ:181-354) on one 256 x 65536 YUYV frame
whose row c holds chroma c with Y = 0..255.  Written as raw uint8
[65536][256] for scripts/chroma_model.c.

usage: python scripts/chroma_masks.py OUT.bin [n_ranges]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from gpu_util import BENCH_RANGES  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    out = sys.argv[1]
    rs = BENCH_RANGES[:int(sys.argv[2])] if len(sys.argv) > 2 else BENCH_RANGES
    W, H = 256, 65536
    j = np.arange(128, dtype=np.uint32)
    c = np.arange(65536, dtype=np.uint32)
    words = (2 * j)[None, :] | ((c & 255)[:, None] << 8) | ((2 * j + 1)[None, :] << 16) | ((c >> 8)[:, None] << 24)
    fr = words.astype("<u4").view(np.uint8).reshape(-1)
    _, mask = oracle.frame(fr, W, H, 2 * W, oracle.LAYOUT_YUYV, rs, want_mask=True)
    mask.astype(np.uint8).tofile(out)
    nz = (mask != 0).mean()
    print(f"{out}: {mask.shape}, nonzero pixels {nz:.4f}, distinct masks {np.unique(mask).tolist()}")


if __name__ == "__main__":
    main()
