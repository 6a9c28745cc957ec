"""Diagnose: import trik_hsv (loads /opt/rocm's HIP runtime) BEFORE torch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import trik_hsv  # noqa: E402
import torch  # noqa: E402

maps = open("/proc/self/maps").read().split("\n")
print("\n".join(sorted(set(l.split()[-1] for l in maps if "amdhip" in l or "hsa-runtime" in l))))
print("is_available", torch.cuda.is_available())
try:
    d = trik_hsv.Detector()
    print("create ok")
    d.close()
except Exception as e:  # noqa: BLE001
    print("create failed:", e)
try:
    x = torch.zeros(1, device="cuda")
    print("torch alloc ok")
    d = trik_hsv.Detector()
    print("create after torch alloc ok")
    d.close()
except Exception as e:  # noqa: BLE001
    print("after torch alloc failed:", e)
