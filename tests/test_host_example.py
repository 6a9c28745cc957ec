"""The reference's ARM-side call sequence written in plain C against the
library (examples/host_process.c): it compiles and
links with gcc on the CPU, and on the GPU its targets and preview equal the
oracle's (WSEQ:412-508 via trik_oracle_run)."""
import os
import subprocess
import tempfile
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(d):
    exe = os.path.join(d, "host_process")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples"), f"OUT={d}"], check=True)
    return exe


def test_host_example_builds_and_links():
    with tempfile.TemporaryDirectory() as d:
        exe = _build(d)
        assert os.path.exists(exe)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,kind,rng", [(640, 480, 1, (0, 30, 50, 100, 30, 100)),
                                          (320, 240, 0, (330, 20, 30, 100, 30, 100))])
def test_host_example_matches_oracle(oracle_mod, w, h, kind, rng):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    frame = oracle_mod.synth(1, w, h, 2 * w, oracle_mod.LAYOUT_YUYV, kind, 0x7A1C, first_frame=5)
    with tempfile.TemporaryDirectory() as d:
        exe = _build(d)
        path = os.path.join(d, "frame.yuyv")
        frame.tofile(path)
        res = subprocess.run([exe, path, str(w), str(h)] + [str(v) for v in rng], capture_output=True,
                             text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    rc, tx, ty, ts, crc = res.stdout.split()
    _, oa, pv = oracle_mod.run(frame, w, h, 2 * w, oracle_mod.LAYOUT_YUYV, rng, out_width=w // 2,
                               out_height=h // 2, out_line_length=w)
    assert (int(rc), int(tx), int(ty), int(ts)) == (0, oa["target_x"], oa["target_y"], oa["target_size"])
    assert int(crc, 16) == zlib.crc32(np.ascontiguousarray(pv).tobytes())
