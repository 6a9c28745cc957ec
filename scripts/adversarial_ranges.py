"""Chroma-run vs stripe kernel time for range sets of increasing exact-path
share (uniform C3 frames), to place the AUTO selector's threshold.

usage (GPU box): python scripts/adversarial_ranges.py [frames]
Prints one line per range set: the builder's expected flagged-word share, the
kernel each hot-kernel setting ran, and its ms per batch.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import trik_hsv  # noqa: E402

SETS = {
    "bench 4 ranges": [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
                       (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)],
    "hue slivers": [(10, 12, 10, 100, 10, 100), (100, 102, 10, 100, 10, 100),
                    (200, 202, 10, 100, 10, 100), (300, 302, 10, 100, 10, 100)],
    "two S bands": [(0, 359, 20, 30, 0, 100), (0, 359, 60, 70, 0, 100)],
    "four V bands": [(0, 359, 0, 100, 20, 25), (0, 359, 0, 100, 40, 45),
                     (0, 359, 0, 100, 60, 65), (0, 359, 0, 100, 80, 85)],
    "four S bands": [(0, 359, 20, 25, 0, 100), (0, 359, 40, 45, 0, 100),
                     (0, 359, 60, 65, 0, 100), (0, 359, 80, 85, 0, 100)],
    "one V range": [(0, 359, 0, 100, 30, 70)],
    "S+V hue-free": [(0, 359, 30, 100, 20, 100), (0, 359, 0, 100, 60, 100)],
}


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    W, H = 640, 480
    ll = 2 * W
    dev = torch.device("cuda", 0)
    frames = torch.empty(F * H * ll, dtype=torch.uint8, device=dev)
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, 0, 0x7A1C)
    stream = torch.cuda.current_stream()
    for name, ranges in SETS.items():
        det = trik_hsv.Detector()
        sums = torch.zeros((F, len(ranges), 3), dtype=torch.int64, device=dev)
        line = [f"{name:16s}"]
        for hot in (trik_hsv.HOT_CHROMA, trik_hsv.HOT_STRIPE, trik_hsv.HOT_AUTO):
            det.set_hot_kernel(hot)
            det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
            if hot == trik_hsv.HOT_CHROMA:
                line.append(f"flagged {det.chroma_flagged_share():.3f}")
            for _ in range(10):  # the clocks ramp
                det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ran = {trik_hsv.HOT_CHROMA: "chroma", trik_hsv.HOT_STRIPE: "stripe"}.get(det.last_hot_kernel(), "?")
            ms = e0.elapsed_time(e1) / 20
            frac = F * H * ll / (ms * 1e-3) / 8e12
            line.append(f"{['auto', 'stripe', 'chroma', 'generic'][hot] if hot < 4 else hot}->{ran} "
                        f"{ms:.3f} ms ({100 * frac:.1f} %)")
        det.close()
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
