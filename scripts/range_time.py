"""Auto-range batch timing on two inputs (development timing of the in-tree
library variant): the synthetic scene of bench_operator.py and uniform random
bytes (every lane of a wave on its own H/S/V bin -- the worst case for the
wave-peeled histogram atomics).  usage: python scripts/range_time.py [--frames N] [--only scene|random]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trik-media-sensors-dsp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--only", choices=["scene", "random"], default=None)
    args = ap.parse_args()
    import torch

    import trik_hsv
    W, H, LL, F = 640, 480, 1280, args.frames
    dev = torch.empty(F * H * LL, dtype=torch.uint8, device="cuda")
    out = {"lib": "in-tree"}
    for name in ((args.only,) if args.only else ("scene", "random")):
        if name == "scene":
            trik_hsv.synth(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, 1, 0x7A1C)
        else:
            dev.random_(0, 256)
        res = None
        for _ in range(3):
            res = trik_hsv.batch_auto_range(dev, W, H, LL, trik_hsv.LAYOUT_YUYV)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(10):
            trik_hsv.batch_auto_range(dev, W, H, LL, trik_hsv.LAYOUT_YUYV)
        ev1.record()
        torch.cuda.synchronize()
        out[name] = {"ms": round(ev0.elapsed_time(ev1) / 10, 4),
                     "check": int(res.to(torch.int64).sum().item()) if hasattr(res, "to") else str(res)[:40]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
