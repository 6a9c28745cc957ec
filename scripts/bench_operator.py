"""Measure the operator outputs of SURVEY 8(f) rows 1-2 on the C3 batch.

  preview     trik_hsv_batch_preview: 4096 x 640x480 YUYV -> 320x240 RGB565X
              previews for one range.  Algorithmic bytes per frame: the source
              rows the 2:1 preview samples (H/2 rows of lineLength bytes) plus
              the preview written (outH * outLineLength), read/written once.
  auto_range  trik_hsv_batch_auto_range: the central zone of each frame
              (159 x 159 px at 640x480, 2 B/px) -- small, launch/latency-bound.
  line        trik_hsv_line_batch: 4096 x 640x480 ov7670 (YUV422P) frames, the
              line sensor's sums + OutArgs; algorithmic bytes = both planes
              (2 B/px) once.  line_preview: its 320x240 previews.
  blob        trik_hsv_blob_batch: 4096 x 640x480 ov7670 frames through the
              multi-blob sensor (metapixel bitmap + clusterer + 8 targets).
  process     one host frame through the XDAIS quartet (H2D + kernels + D2H,
              PCIe-inclusive latency per frame), with preview and auto range.

Prints one JSON object.  usage: python scripts/bench_operator.py [--frames N]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TRIK_HSV_PKG_DIR: a directory holding another build's trik_hsv package (A/B)
sys.path.insert(0, os.environ.get("TRIK_HSV_PKG_DIR", os.path.join(ROOT, "trik-media-sensors-dsp_amd")))
HBM_PEAK_GBS = 8000.0


def timed(fn, stream, iters):
    """Average GPU time per call of `iters` back-to-back calls (asynchronous
    launches, so host-side call overhead overlaps the previous call's kernels),
    after `iters` untimed calls of the same operation (the first calls after
    another operation's batches run up to 25 % slower: the auto-range launches
    right after the previews' 1.9 GB of stores took 198 -> 161 us in
    profiles/r06/r06x_operator_kernel_trace_auto_range.txt)."""
    import torch

    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(iters):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true", help="skip the oracle CPU baselines")
    args = ap.parse_args()
    import numpy as np
    import torch

    import trik_hsv

    W, H, LL, F = 640, 480, 1280, args.frames
    OW, OH, OLL = 320, 240, 640
    T0 = (0, 30, 50, 100, 30, 100)
    dev = torch.empty(F * H * LL, dtype=torch.uint8, device="cuda")
    trik_hsv.synth(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, 1, 0x7A1C)
    stream = torch.cuda.current_stream()
    det = trik_hsv.Detector()
    sums, _ = det.process_batch(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, [T0])
    out = {}

    pv_ms = timed(lambda: det.batch_preview(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, T0, sums,
                                            out_width=OW, out_height=OH, out_line_length=OLL),
                  stream, args.iters)
    pv_bytes = F * ((H // 2) * LL + OH * OLL)
    out["preview"] = {"frames": F, "ms": round(pv_ms, 4), "Mframes_per_s": round(F / pv_ms / 1e3, 3),
                      "bytes_algorithmic": pv_bytes,
                      "achieved_GBs": round(pv_bytes / (pv_ms / 1e3) / 1e9, 1),
                      "hbm_frac": round(pv_bytes / (pv_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                      "note": "preview_rows2_kernel (the 2:1 map: writes every preview byte, guide lines included) + overlay_kernel (the target circle)"}

    ar_ms = timed(lambda: trik_hsv.batch_auto_range(dev, W, H, LL, trik_hsv.LAYOUT_YUYV), stream,
                  args.iters)
    zone = 159 * 159
    out["auto_range"] = {"frames": F, "ms": round(ar_ms, 4), "Mframes_per_s": round(F / ar_ms / 1e3, 3),
                         "zone_px_per_frame": zone,
                         "achieved_GBs": round(F * zone * 2 / (ar_ms / 1e3) / 1e9, 1)}

    lf = min(F, 4096)
    lfb = 2 * H * W
    ldev = torch.empty(lf * lfb, dtype=torch.uint8, device="cuda")
    trik_hsv.synth(ldev, W, H, W, trik_hsv.LAYOUT_OV7670, 1, 0x7A1C)
    ln_ms = timed(lambda: trik_hsv.line_batch(ldev, W, H, W, 0, 30), stream, args.iters)
    out["line"] = {"frames": lf, "ms": round(ln_ms, 4), "Mframes_per_s": round(lf / ln_ms / 1e3, 3),
                   "bytes_algorithmic": lf * lfb,
                   "achieved_GBs": round(lf * lfb / (ln_ms / 1e3) / 1e9, 1),
                   "hbm_frac": round(lf * lfb / (ln_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                   "note": "line_vec_kernel + line_targets_kernel"}
    lsums, _ = trik_hsv.line_batch(ldev, W, H, W, 0, 30)
    lp_ms = timed(lambda: det.line_preview(ldev, W, H, W, 0, 30, lsums, out_width=OW, out_height=OH,
                                           out_line_length=OLL), stream, args.iters)
    lp_bytes = lf * (H // 2 * 2 * W + OH * OLL)
    out["line_preview"] = {"frames": lf, "ms": round(lp_ms, 4),
                           "achieved_GBs": round(lp_bytes / (lp_ms / 1e3) / 1e9, 1),
                           "hbm_frac": round(lp_bytes / (lp_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    RED = (0, 20, 80, 20, 50, 50)
    bl_ms = timed(lambda: det.blob_batch(ldev, W, H, W, RED), stream, args.iters)
    out["blob"] = {"frames": lf, "ms": round(bl_ms, 4), "Mframes_per_s": round(lf / bl_ms / 1e3, 3),
                   "achieved_GBs": round(lf * lfb / (bl_ms / 1e3) / 1e9, 1),
                   "hbm_frac": round(lf * lfb / (bl_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                   "note": "bitmap (blob_chroma_meta_kernel for large batches, else blob_meta_kernel) + blob_ccl_kernel (one wave per frame)"}
    ldev_host = ldev[: 8 * lfb].cpu().numpy()
    del ldev

    s = trik_hsv.ObjectSensor()
    assert s.set_params(W, H, LL) == 0
    host = dev[: H * LL].cpu().numpy()
    prev = np.zeros(OH * OLL, np.uint8)
    for _ in range(3):
        s.process(host, T0, out_buffer=prev, auto_detect=True)
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        rc, _ = s.process(host, T0, out_buffer=prev, auto_detect=True)
        assert rc == 0
    dt = (time.perf_counter() - t0) / n
    out["process_single_frame"] = {"ms_per_frame": round(dt * 1e3, 4),
                                   "note": "host frame in, preview + targets + detect* out; "
                                           "PCIe-inclusive, one synchronous call per frame"}
    s.close()
    det.close()
    if not args.no_cpu:
        cpu_baselines(out, dev, ldev_host, W, H, LL, OW, OH, OLL, T0)
    print(json.dumps(out))


def cpu_baselines(out, dev, ldev_host, W, H, LL, OW, OH, OLL, T0):
    """The oracle (C restatement of the reference, one thread) on a few of the
    same frames, per row: ms per frame, beside the GPU's ms per frame."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    oracle.build()
    n = 8
    fb = H * LL
    frames = dev[: n * fb].cpu().numpy()
    lfb = 2 * H * W
    lframes = ldev_host[: n * lfb]

    def per_frame(fn):
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        return (time.perf_counter() - t0) / n * 1e3

    rows = {
        "preview": lambda i: oracle.run(frames[i * fb:(i + 1) * fb], W, H, LL, 0, T0, out_width=OW,
                                        out_height=OH, out_line_length=OLL),
        "auto_range": lambda i: oracle.run(frames[i * fb:(i + 1) * fb], W, H, LL, 0, T0, auto_detect=True,
                                           preview=False),
        "line": lambda i: oracle.line_run(lframes[i * lfb:(i + 1) * lfb], W, H, W, 0, 30, preview=False),
        "blob": lambda i: oracle.blob_run(lframes[i * lfb:(i + 1) * lfb], W, H, W, hsv=(0, 20, 80, 20, 50, 50),
                                          preview=False),
    }
    for k, fn in rows.items():
        ms = per_frame(fn)
        gpu_ms = out[k]["ms"] / out[k]["frames"]
        out[k]["cpu_baseline"] = {"kind": "port", "cores": 1, "ms_per_frame": round(ms, 3),
                                  "sample": f"{n} frames of the same batch, oracle (whole run incl. its "
                                            "per-pixel HSV pass), single thread",
                                  "gpu_ms_per_frame": round(gpu_ms, 6),
                                  "gpu_over_cpu": round(ms / gpu_ms, 1)}


if __name__ == "__main__":
    main()
