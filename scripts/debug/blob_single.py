"""One VGA frame through the multi-blob codec, N times (for kernel traces)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import trik_hsv  # noqa: E402

fr = oracle.blob_scene(640, 480, 640, 1, noise=0.01)
prev = np.zeros(240 * 640, np.uint8)
b = trik_hsv.BlobSensor()
b.set_params(640, 480, 640)
for _ in range(50):
    rc, _ = b.process(fr, (0, 20, 80, 20, 50, 50), out_buffer=prev)
    assert rc == 0
b.close()
print("ok")
