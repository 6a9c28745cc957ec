"""Handles from several host threads (handles are
independent; calls on one handle are serialised by its mutex), and the batched
API on a non-default stream.  Results must equal the oracle's regardless."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T0 = (0, 30, 50, 100, 30, 100)
T3 = (330, 20, 30, 100, 30, 100)


@pytest.fixture(scope="module")
def hsv():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import trik_hsv

    return trik_hsv


def test_threads_own_and_shared_handles(hsv, oracle_mod):
    w, h, ll = 320, 240, 640
    frames = [oracle_mod.synth(1, w, h, ll, 0, 1, 0x7A1C, first_frame=i) for i in range(6)]
    want = {}
    for i, fr in enumerate(frames):
        for rng in (T0, T3):
            _, oa, pv = oracle_mod.run(fr, w, h, ll, 0, rng, out_width=160, out_height=120, out_line_length=320)
            want[(i, rng)] = ((oa["target_x"], oa["target_y"], oa["target_size"]), pv)
    shared = hsv.ObjectSensor()
    assert shared.set_params(w, h, ll, out_width=160, out_height=120, out_line_length=320) == 0
    errors = []

    def worker(seed, use_shared):
        s = shared if use_shared else hsv.ObjectSensor()
        try:
            if not use_shared:
                assert s.set_params(w, h, ll, out_width=160, out_height=120, out_line_length=320) == 0
            rs = np.random.default_rng(seed)
            for _ in range(20):
                i = int(rs.integers(0, len(frames)))
                rng = T0 if rs.integers(0, 2) else T3
                out = np.zeros(120 * 320, np.uint8)
                rc, oa = s.process(frames[i], rng, out_buffer=out)
                t, pv = want[(i, rng)]
                if rc != 0 or (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) != t or not np.array_equal(out, pv):
                    errors.append((seed, i, rng))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
        finally:
            if not use_shared:
                s.close()

    threads = [threading.Thread(target=worker, args=(k, k % 2 == 0)) for k in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    shared.close()
    assert not errors, errors[:5]


def test_batch_api_on_a_side_stream(hsv, oracle_mod):
    import torch

    w, h, ll, n = 640, 480, 1280, 8
    host = oracle_mod.synth(n, w, h, ll, 0, 0, 0x7A1C, first_frame=100)
    side = torch.cuda.Stream()
    det = hsv.Detector()
    try:
        with torch.cuda.stream(side):
            dev = torch.from_numpy(host).cuda()
            sums, targets = det.process_batch(dev, w, h, ll, 0, [T0, T3], stream=side)
        side.synchronize()
        want_s, want_t = oracle_mod.batch(host, h * ll, n, w, h, ll, 0, [T0, T3])
        assert np.array_equal(sums.cpu().numpy(), want_s)
        assert np.array_equal(targets[:, :, :3].cpu().numpy(), want_t)
    finally:
        det.close()


def test_import_order_one_hip_runtime(hsv):
    """`import trik_hsv` before `import torch` in a fresh interpreter: the
    package binds the library to torch's HIP runtime."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import trik_hsv; import torch; "
            "d = trik_hsv.Detector(); d.close(); print('ok')" % os.path.join(root, "trik-media-sensors-dsp_amd"))
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0 and "ok" in res.stdout, res.stderr[-2000:]
