"""GPU time of trik_hsv_blob_batch (4096 ov7670 VGA frames, scene or uniform)
of the in-tree library.  usage: python scripts/blob_time.py [frames] [kind]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import trik_hsv  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
kind = int(sys.argv[2]) if len(sys.argv) > 2 else 1
W, H = 640, 480
dev = torch.empty(F * 2 * H * W, dtype=torch.uint8, device="cuda")
trik_hsv.synth(dev, W, H, W, trik_hsv.LAYOUT_OV7670, kind, 0x7A1C)
det = trik_hsv.Detector()
s = torch.cuda.current_stream()
RED = (0, 20, 80, 20, 50, 50)
det.blob_batch(dev, W, H, W, RED, stream=s)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
for _ in range(10):
    det.blob_batch(dev, W, H, W, RED, stream=s)
b.record(s)
torch.cuda.synchronize()
print(f"frames {F} kind {kind}: {a.elapsed_time(b) / 10:.3f} ms")
