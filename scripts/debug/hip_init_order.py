"""Diagnose: create a handle after torch.cuda.is_available() but before any
torch CUDA allocation; list the HIP runtimes mapped into the process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
import torch  # noqa: E402

print("is_available", torch.cuda.is_available())
import trik_hsv  # noqa: E402

try:
    d = trik_hsv.Detector()
    print("create ok")
    d.close()
except Exception as e:  # noqa: BLE001
    print("create failed:", e)
maps = open("/proc/self/maps").read().split("\n")
libs = sorted(set(l.split()[-1] for l in maps if "amdhip" in l or "hsa-runtime" in l))
print("\n".join(libs))
x = torch.zeros(1, device="cuda")
try:
    d = trik_hsv.Detector()
    print("create after torch alloc ok")
    d.close()
except Exception as e:  # noqa: BLE001
    print("create after torch alloc failed:", e)
