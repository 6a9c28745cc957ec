"""Per-launch GPU time of the hot path on C3, several ways, in one process
(development only): the hot kernel alone (trik_hsv_batch_sums, adding into
sums) and the fused full step (trik_hsv_process_batch_totals), each enqueued
back to back (as bench.py does) and synchronised after every launch (as
scripts/kbench does).

usage (GPU box): python scripts/step_timing.py [reps]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import trik_hsv  # noqa: E402

RANGES = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
          (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    F, W, H = 4096, 640, 480
    ll = 2 * W
    frames = torch.empty(F * H * ll, dtype=torch.uint8, device="cuda")
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, 0, 0x7A1C)
    det = trik_hsv.Detector(hot=trik_hsv.HOT_CHROMA)
    sums = torch.zeros((F, 4, 3), dtype=torch.int64, device="cuda")
    targets = torch.zeros((F, 4, 4), dtype=torch.int8, device="cuda")
    totals = torch.zeros((4, 3), dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()

    def hot():
        det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, RANGES, sums, stream=stream)

    def full():
        det.process_batch_totals(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, RANGES, sums=sums, targets=targets,
                                 totals=totals, stream=stream)

    def timed(fn, sync):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        for a, b in evs:
            a.record(stream)
            fn()
            b.record(stream)
            if sync:
                b.synchronize()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        return sum(ms) / len(ms), ms[len(ms) // 2]

    for rnd in range(2):
        for name, fn in (("hot kernel (batch_sums)", hot), ("fused step (process_batch_totals)", full)):
            for sync in (False, True):
                avg, med = timed(fn, sync)
                print(f"round {rnd}  {name:36s} {'sync each' if sync else 'back to back':12s} "
                      f"avg {avg:.4f} ms  median {med:.4f} ms", flush=True)
    det.close()


if __name__ == "__main__":
    main()
