"""A/B timing of the multi-blob pipeline (trik_hsv_blob_batch, 4096 ov7670 VGA
frames) or of autoDetectHsv (--what range: trik_hsv_batch_auto_range, 4096
YUYV VGA frames) across library variants (development only; GPU box).

usage: python scripts/blob_ab.py [--what blob|range] [--frames N] [--reps R] lib1 [lib2 ...]
  libs: paths to libtrik_hsv.so variants (e.g. trik-media-sensors-dsp_amd/ab/x/libtrik_hsv.so)

Each variant runs in its own process on a private copy of the host package
with the variant as its library; kinds 0 (uniform bytes: dense bitmaps) and 1
(scene) are timed with HIP events (median of R rounds of 5 batches), and the
results of every variant are compared with the first one's (top clusters and
label counts)."""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "trik-media-sensors-dsp_amd", "trik_hsv")

CHILD = r"""
import hashlib, json, sys
import torch
import trik_hsv
F, reps = int(sys.argv[1]), int(sys.argv[2])
W, H = 640, 480
RED = (0, 20, 80, 20, 50, 50)
dev = torch.empty(F * 2 * H * W, dtype=torch.uint8, device="cuda")
det = trik_hsv.Detector()
s = torch.cuda.current_stream()
res = {}
for kind in (0, 1):
    trik_hsv.synth(dev, W, H, W, trik_hsv.LAYOUT_OV7670, kind, 0x7A1C)
    out = det.blob_batch(dev, W, H, W, RED, stream=s)
    torch.cuda.synchronize()
    digest = hashlib.sha256(out["top"].cpu().numpy().tobytes() + out["n_labels"].cpu().numpy().tobytes()).hexdigest()[:16]
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(5):
            det.blob_batch(dev, W, H, W, RED, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b) / 5)
    t.sort()
    res[kind] = {"ms": round(t[len(t) // 2], 4), "min": round(t[0], 4), "digest": digest,
                 "labels_mean": float(out["n_labels"].float().mean())}
print(json.dumps(res))
"""


CHILD_RANGE = r"""
import hashlib, json, sys
import torch
import trik_hsv
F, reps = int(sys.argv[1]), int(sys.argv[2])
W, H, LL = 640, 480, 1280
dev = torch.empty(F * H * LL, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
res = {}
for kind in (0, 1):
    if kind == 1:
        trik_hsv.synth(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, 1, 0x7A1C)
    else:
        trik_hsv.synth(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, 0, 0x7A1C)
    out = trik_hsv.batch_auto_range(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, stream=s)
    torch.cuda.synchronize()
    digest = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(5):
            trik_hsv.batch_auto_range(dev, W, H, LL, trik_hsv.LAYOUT_YUYV, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b) / 5)
    t.sort()
    res[kind] = {"ms": round(t[len(t) // 2], 4), "min": round(t[0], 4), "digest": digest, "labels_mean": 0}
print(json.dumps(res))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["blob", "range"], default="blob")
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    rows = []
    for lib in a.libs:
        with tempfile.TemporaryDirectory() as d:
            shutil.copytree(PKG, os.path.join(d, "trik_hsv"), ignore=shutil.ignore_patterns("*.so", "__pycache__"))
            shutil.copy(lib, os.path.join(d, "trik_hsv", "libtrik_hsv.so"))
            env = dict(os.environ, PYTHONPATH=d)
            r = subprocess.run([sys.executable, "-c", CHILD if a.what == "blob" else CHILD_RANGE, str(a.frames), str(a.reps)], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(lib, "FAILED", r.stderr[-2000:], flush=True)
                sys.exit(r.returncode)
            res = json.loads(r.stdout.strip().splitlines()[-1])
        rows.append((lib, res))
        same = "" if len(rows) == 1 else "  " + " ".join(
            f"k{k}:{'same' if res[k]['digest'] == rows[0][1][k]['digest'] else 'DIFF'}" for k in res)
        print(f"{lib}: uniform {res['0']['ms']:.4f} ms (min {res['0']['min']:.4f}, labels {res['0']['labels_mean']:.0f}), "
              f"scene {res['1']['ms']:.4f} ms (min {res['1']['min']:.4f}){same}", flush=True)


if __name__ == "__main__":
    main()
