"""Per-call latency of the XDAIS process() path (one host VGA frame per call),
for the three codecs and with/without preview and auto range.  Prints JSON.
usage: python scripts/debug/process_latency.py [--calls N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch

    import trik_hsv

    W, H = 640, 480
    rng = np.random.default_rng(1)
    yuyv = rng.integers(0, 256, H * W * 2, dtype=np.uint8)
    planes = rng.integers(0, 256, 2 * H * W, dtype=np.uint8)
    prev = np.zeros(240 * 640, np.uint8)
    T0 = (0, 30, 50, 100, 30, 100)
    out = {}

    def run(name, fn):
        for _ in range(5):
            fn()
        t0 = time.perf_counter()
        for _ in range(args.calls):
            rc = fn()
            assert rc == 0
        out[name] = round((time.perf_counter() - t0) / args.calls * 1e3, 4)

    s0 = trik_hsv.ObjectSensor(trik_hsv._default_params(0))
    s0.set_params(W, H, 2 * W)
    run("ball_targets_only", lambda: s0.process(yuyv, T0)[0])
    s0.close()
    s = trik_hsv.ObjectSensor()
    s.set_params(W, H, 2 * W)
    run("ball_preview", lambda: s.process(yuyv, T0, out_buffer=prev)[0])
    run("ball_preview_auto", lambda: s.process(yuyv, T0, out_buffer=prev, auto_detect=True)[0])
    s.close()
    ln = trik_hsv.LineSensor()
    ln.set_params(W, H, W, out_width=320, out_height=240, out_line_length=640)
    run("line_preview", lambda: ln.process(planes, (0, 359, 0, 100, 0, 30), out_buffer=prev)[0])
    ln.close()
    b = trik_hsv.BlobSensor()
    b.set_params(W, H, W)
    run("blob_preview", lambda: b.process(planes, (0, 20, 80, 20, 50, 50), out_buffer=prev)[0])
    b.close()
    # raw copies for reference: pageable H2D of one frame, D2H of one preview
    d = torch.empty(H * W * 2, dtype=torch.uint8, device="cuda")
    t = torch.from_numpy(yuyv)
    run("h2d_pageable_614KB", lambda: (d.copy_(t), torch.cuda.synchronize(), 0)[2])
    tp = t.pin_memory()
    run("h2d_pinned_614KB", lambda: (d.copy_(tp, non_blocking=True), torch.cuda.synchronize(), 0)[2])
    print(json.dumps({"ms_per_call": out, "calls": args.calls}))


if __name__ == "__main__":
    main()
