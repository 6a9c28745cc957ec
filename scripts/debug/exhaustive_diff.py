"""Debug aid: where does the hot kernel's per-pixel mask differ from the oracle
over all 2^24 YUV triples?  Prints counts and sample triples with the oracle's
intermediate values.  usage (GPU box): python scripts/debug/exhaustive_diff.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "trik-media-sensors-dsp_amd")]
import torch  # noqa: E402

import oracle  # noqa: E402
import trik_hsv  # noqa: E402
from gpu_util import BENCH_RANGES, exhaustive_yuyv_frame  # noqa: E402

frame, w, h, ll = exhaustive_yuyv_frame()
tab = oracle.yuv_table(closed=False)
det = trik_hsv.Detector()
dev = torch.from_numpy(frame).cuda()
for name, ranges in [("full", [(0, 359, 0, 100, 0, 100)]), ("bench", BENCH_RANGES)]:
    _, want = oracle.frame(frame, w, h, ll, 0, ranges, want_mask=True)
    masks, _ = det.batch_masks(dev, w, h, ll, 0, ranges)
    got = masks[0].cpu().numpy()
    bad = np.argwhere(got != want)
    print(f"[{name}] {len(bad)} of {got.size} pixels differ; got-bits {int(np.unpackbits(got.astype(np.uint8)).sum())} "
          f"want-bits {int(np.unpackbits(want.astype(np.uint8)).sum())}")
    words = frame.view("<u4").reshape(h, w // 2)
    for (yy, xx) in bad[:12]:
        wd = int(words[yy, xx // 2])
        Y = (wd >> (16 * (xx & 1))) & 255
        U, V = (wd >> 8) & 255, wd >> 24
        e = int(tab[Y | (U << 8) | (V << 16)])
        rgb, hsv = e >> 32, e & 0xFFFFFFFF
        print(f"  x={xx} y={yy} YUV=({Y},{U},{V}) rgb=({rgb & 255},{rgb >> 8 & 255},{rgb >> 16 & 255}) "
              f"hsv=({hsv & 255},{hsv >> 8 & 255},{hsv >> 16 & 255}) want={want[yy, xx]:#x} got={got[yy, xx]:#x}")
    if len(bad):
        xs = bad[:, 1]
        print("  column mod 8 histogram:", np.bincount(xs % 8, minlength=8).tolist(),
              " lane-ish (x//8 %32):", np.bincount((xs // 8) % 32, minlength=32).tolist()[:8], "...")
det.close()
