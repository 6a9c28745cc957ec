"""Host-side cost of one warm full step (development only): the Python call
(Detector.process_batch_totals) and the C-ABI call alone, enqueue only.

usage (GPU box): python scripts/host_cost.py
"""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import trik_hsv  # noqa: E402

RANGES = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
          (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]


def main():
    F, W, H = 4096, 640, 480
    ll = 2 * W
    frames = torch.empty(F * H * ll, dtype=torch.uint8, device="cuda")
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, 0, 0x7A1C)
    det = trik_hsv.Detector()
    sums = torch.zeros((F, 4, 3), dtype=torch.int64, device="cuda")
    targets = torch.zeros((F, 4, 4), dtype=torch.int8, device="cuda")
    totals = torch.zeros((4, 3), dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    for _ in range(30):
        det.process_batch_totals(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, RANGES, sums=sums, targets=targets,
                                 totals=totals, stream=stream)
    torch.cuda.synchronize()
    for n in (8, 32):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            det.process_batch_totals(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, RANGES, sums=sums, targets=targets,
                                     totals=totals, stream=stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"python call x{n}: enqueue {1e6 * (t1 - t0) / n:.1f} us/call, wall {1e6 * (t2 - t0) / n:.1f} us/step",
              flush=True)
    # one step after an idle GPU: host enqueue to completion
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        det.process_batch_totals(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, RANGES, sums=sums, targets=targets,
                                 totals=totals, stream=stream)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"single step from idle: enqueue {1e6 * (t1 - t0):.1f} us, wall {1e6 * (t2 - t0):.1f} us", flush=True)
    det.close()


if __name__ == "__main__":
    main()
