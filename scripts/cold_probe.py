"""A few cold batches (range sets new to a warm handle), synchronised, for a
trace of where the cold step's time goes (development only).

usage (GPU box): rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace ... -- python3 scripts/cold_probe.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# argv[1]: a directory holding another copy of the trik_hsv package (A/B runs)
sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import trik_hsv  # noqa: E402

BENCH = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
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

    def call(rs):
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        c0.record(stream)
        h0 = time.perf_counter()
        det.process_batch_totals(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, rs, sums=sums, targets=targets,
                                 totals=totals, stream=stream)
        h1 = time.perf_counter()
        c1.record(stream)
        torch.cuda.synchronize()
        return c0.elapsed_time(c1), (h1 - h0) * 1e3

    for j in range(12):
        rs = [(BENCH[0][0] + j,) + BENCH[0][1:]] + BENCH[1:]
        cold, cold_host = call(rs)
        warm, _ = call(rs)
        warm2, _ = call(rs)
        print(f"set {j}: cold {cold:.4f} ms (host {cold_host:.4f})  next {warm:.4f}  next {warm2:.4f}", flush=True)
    det.close()


if __name__ == "__main__":
    main()
