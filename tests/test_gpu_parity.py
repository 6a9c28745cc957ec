"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact everywhere (the path is integer arithmetic plus one IEEE fp32
sqrt/div/ceil in the epilogue, which must also match exactly).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from gpu_util import (BENCH_RANGES, LAYOUT_OV7670, LAYOUT_YUYV, T0, T1, T2, T3,
                      exhaustive_yuyv_frame, sums_from_mask)

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.json")

EDGE_RANGES = [
    (0, 359, 0, 100, 0, 100),      # full
    (10, 10, 100, 100, 100, 100),  # single point
    (2, 1, 0, 100, 0, 100),        # wrap, From == To + 1 after scaling
    (359, 0, 20, 100, 20, 100),    # wrap through 0
    (400, 500, 200, 250, 0, 255),  # out-of-range args, clamped
    (0, 359, 0, 0, 0, 100),        # grey only
    (0, 359, 0, 100, 0, 10),       # dark only
    (120, 120, 0, 100, 0, 100),    # From == To
]


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def hsv():
    import trik_hsv

    return trik_hsv


@pytest.fixture(scope="module")
def detector(hsv, torch_dev):
    d = hsv.Detector()
    yield d
    d.close()


def _to_dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


def test_library_is_native(hsv):
    assert "gfx950" in hsv.version()


@pytest.mark.parametrize("group", ["bench", "edge"])
def test_exhaustive_all_yuv_triples(torch_dev, detector, oracle_mod, group):
    """Every (Y,U,V) triple through the hot kernel (verification mode) vs the oracle."""
    torch = torch_dev
    ranges = BENCH_RANGES + EDGE_RANGES[:4] if group == "bench" else EDGE_RANGES
    frame, w, h, ll = exhaustive_yuyv_frame()
    _, want = oracle_mod.frame(frame, w, h, ll, LAYOUT_YUYV, ranges, want_mask=True)
    dev = _to_dev(torch, frame)
    masks, sums = detector.batch_masks(dev, w, h, ll, LAYOUT_YUYV, ranges)
    got = masks[0].cpu().numpy()
    bad = np.count_nonzero(got != want)
    assert bad == 0, f"{bad} pixels differ; first at {np.argwhere(got != want)[:5].tolist()}"
    assert sums[0].cpu().numpy().tolist() == sums_from_mask(want, len(ranges)).tolist()


def test_exhaustive_ov7670_layout(torch_dev, detector, oracle_mod):
    """Same 2^24 triples through the ov7670 semi-planar layout."""
    torch = torch_dev
    frame, w, h, ll = exhaustive_yuyv_frame()
    px = frame.reshape(h, w // 2, 4)
    ylum = np.stack([px[..., 0], px[..., 2]], -1).reshape(h, w)
    chroma = np.stack([px[..., 3], px[..., 1]], -1).reshape(h, w)  # even = V, odd = U
    planar = np.concatenate([ylum.reshape(-1), chroma.reshape(-1)])
    _, want = oracle_mod.frame(planar, w, h, w, LAYOUT_OV7670, BENCH_RANGES, want_mask=True)
    masks, _ = detector.batch_masks(_to_dev(torch, planar), w, h, w, LAYOUT_OV7670, BENCH_RANGES)
    assert np.array_equal(masks[0].cpu().numpy(), want)


def test_golden_frames(torch_dev, hsv, detector):
    torch = torch_dev
    with open(GOLDEN) as f:
        g = json.load(f)
    for c in g["cases"]:
        w, h, ll, lay = c["width"], c["height"], c["line_length"], c["layout"]
        fb = hsv.frame_bytes(w, h, ll, lay)
        dev = torch.zeros(max(fb, 16), dtype=torch.uint8, device="cuda")
        if fb:
            hsv.synth(dev, w, h, ll, lay, c["kind"], c["seed"], first_frame=c["frame"], n_frames=1)
            assert hashlib.sha256(dev[:fb].cpu().numpy().tobytes()).hexdigest() == c["frame_sha256"], c["name"]
        rs = [g["ranges"][r] for r in c["ranges"]]
        sums, tg = detector.process_batch(dev, w, h, ll, lay, rs, n_frames=1, frame_stride=max(fb, 16))
        assert sums[0].cpu().numpy().tolist() == c["sums"], c["name"]
        assert tg[0, :, :3].cpu().numpy().tolist() == c["targets"], c["name"]


@pytest.mark.parametrize("w,h,layout,kind,ranges,n", [
    (640, 480, LAYOUT_YUYV, 0, BENCH_RANGES, 24),          # C3 shape, uniform
    (640, 480, LAYOUT_YUYV, 1, BENCH_RANGES, 24),          # C3 shape, scene
    (1280, 720, LAYOUT_YUYV, 1, [T0, T1], 8),              # C4 shape
    (320, 240, LAYOUT_OV7670, 1, [T0], 16),                # C1 layout
    (640, 480, LAYOUT_YUYV, 0, BENCH_RANGES + EDGE_RANGES, 4),  # 12 ranges = 3 launches
])
def test_batch_vs_oracle(torch_dev, hsv, detector, oracle_mod, w, h, layout, kind, ranges, n):
    torch = torch_dev
    ll = 2 * w if layout == LAYOUT_YUYV else w
    fb = hsv.frame_bytes(w, h, ll, layout)
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, layout, kind, 0x7A1C, first_frame=100)
    host = oracle_mod.synth(n, w, h, ll, layout, kind, 0x7A1C, first_frame=100)
    assert np.array_equal(dev.cpu().numpy(), host)
    sums, tg = detector.process_batch(dev, w, h, ll, layout, ranges)
    want_s, want_t = oracle_mod.batch(host, fb, n, w, h, ll, layout, ranges, n_threads=8)
    assert np.array_equal(sums.cpu().numpy(), want_s)
    assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t)


def test_ragged_and_unaligned(torch_dev, hsv, detector, oracle_mod):
    """lineLength padding, odd frame stride and a misaligned base (byte-load path)."""
    torch = torch_dev
    for (w, h, ll, lay) in [(64, 8, 160, LAYOUT_YUYV), (96, 12, 112, LAYOUT_OV7670),
                            (32, 4, 72, LAYOUT_YUYV), (640, 480, 1344, LAYOUT_YUYV)]:
        fb = hsv.frame_bytes(w, h, ll, lay)
        stride = fb + 3
        n = 5
        host = oracle_mod.synth(n, w, h, ll, lay, 0, 42, frame_stride=stride)
        buf = np.zeros(host.size + 1, np.uint8)
        buf[1:] = host  # base misaligned by one byte
        dev = _to_dev(torch, buf)
        ranges = BENCH_RANGES + EDGE_RANGES[:2]
        sums, tg = detector.process_batch(dev[1:], w, h, ll, lay, ranges, n_frames=n,
                                          frame_stride=stride)
        want_s, want_t = oracle_mod.batch(host, stride, n, w, h, ll, lay, ranges)
        assert np.array_equal(sums.cpu().numpy(), want_s), (w, h, ll, lay)
        assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t), (w, h, ll, lay)
        # aligned copy of the same frames takes the vector-load path
        dev2 = _to_dev(torch, host)
        sums2, _ = detector.process_batch(dev2, w, h, ll, lay, ranges, n_frames=n, frame_stride=stride)
        assert np.array_equal(sums2.cpu().numpy(), want_s)


def test_empty_inputs(torch_dev, detector):
    torch = torch_dev
    dev = torch.zeros(64, dtype=torch.uint8, device="cuda")
    sums, tg = detector.process_batch(dev, 640, 0, 1280, LAYOUT_YUYV, [T0], n_frames=3, frame_stride=0)
    assert sums.abs().sum().item() == 0 and tg.abs().sum().item() == 0
    sums, tg = detector.process_batch(dev, 640, 480, 1280, LAYOUT_YUYV, [T0], n_frames=0)
    assert sums.numel() == 0


def test_rejects_bad_geometry(torch_dev, hsv, detector):
    torch = torch_dev
    dev = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    for (w, h, ll) in [(48, 4, 96), (32, 6, 64), (64, 4, 100)]:
        with pytest.raises(hsv.TrikHsvError):
            detector.process_batch(dev, w, h, ll, LAYOUT_YUYV, [T0], n_frames=1)


def test_epilogue_all_point_counts(torch_dev, hsv, oracle_mod):
    """targets for every N in 0..W*H at 640x480 (centroids spread over the frame)."""
    torch = torch_dev
    w, h = 640, 480
    n = np.arange(0, w * h + 1, dtype=np.int64)
    cx = (n * 7919) % w
    cy = (n * 104729) % h
    sums = np.stack([n, cx * n, cy * n], -1).reshape(-1, 1, 3)
    sums[:, 0, 1] = np.minimum(sums[:, 0, 1], 2**31 - 1)
    sums[:, 0, 2] = np.minimum(sums[:, 0, 2], 2**31 - 1)
    got = hsv.batch_targets(_to_dev(torch, sums), w, h).cpu().numpy()[:, 0, :3]
    idx = np.concatenate([np.arange(0, 5000), np.arange(5000, n.size, 97), [n.size - 1]])
    for i in idx:
        assert tuple(got[i]) == oracle_mod.targets(sums[i, 0], w, h), int(i)


def test_full_c3_batch_properties(torch_dev, hsv, detector, oracle_mod):
    """4096 x 640x480, T=4 (the bench workload): deterministic, and sampled
    frames equal the oracle."""
    torch = torch_dev
    w, h, ll, n = 640, 480, 1280, 4096
    fb = h * ll
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C)
    s1, t1 = detector.process_batch(dev, w, h, ll, LAYOUT_YUYV, BENCH_RANGES)
    s2, t2 = detector.process_batch(dev, w, h, ll, LAYOUT_YUYV, BENCH_RANGES)
    assert torch.equal(s1, s2) and torch.equal(t1, t2)
    s1 = s1.cpu().numpy()
    for f in (0, 1, 2047, 4095):
        host = oracle_mod.synth(1, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C, first_frame=f)
        want, _ = oracle_mod.frame(host, w, h, ll, LAYOUT_YUYV, BENCH_RANGES)
        assert np.array_equal(s1[f], want), f
    assert s1[:, :, 0].min() > 0  # uniform data hits every range in every frame
