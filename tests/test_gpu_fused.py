"""The fused full step (trik_hsv_process_batch_totals): the chroma-run kernel
splits the batch's units evenly over its workgroups, and the wave that counts
a frame's last unit stores the frame's sums and targets; the last workgroup
writes the per-target batch totals -- one launch (trik_hsv_chroma.hip:
chroma_kernel, chroma_fused_ok).

Held to the separate-kernel path (the hot kernel adding into zeroed sums,
then the epilogue and totals kernels) bit for bit, and to the oracle
(oracle/trik_oracle.c: WSEQ:251-354 and the epilogue WSEQ:486-505) on sampled
frames.  Batch sizes that do not divide over the workgroups put a frame's
units in two workgroups (1100, 1000, 257, 40 frames).
"""

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

SEED = 0x7A1C
W, H = 640, 480
LL = 2 * W


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def hsv(torch_dev):
    import trik_hsv

    return trik_hsv


def _frames(torch, hsv, n, kind):
    dev = torch.empty(n * H * LL, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, W, H, LL, LAYOUT_YUYV, kind, SEED)
    return dev


def _separate(torch, hsv, frames, n, ranges):
    """The hot kernel adding into zeroed sums, then the epilogue and totals kernels."""
    det = hsv.Detector(hot=hsv.HOT_CHROMA)
    sums = torch.zeros((n, len(ranges), 3), dtype=torch.int64, device="cuda")
    det.batch_sums(frames, W, H, LL, LAYOUT_YUYV, ranges, sums, n_frames=n, frame_stride=H * LL)
    targets = hsv.batch_targets(sums, W, H)
    totals = hsv.batch_totals_device(sums)
    torch.cuda.synchronize()
    det.close()
    return sums, targets, totals


def _fused(torch, hsv, det, frames, n, ranges):
    # outputs pre-filled with garbage: the fused step writes every element
    sums = torch.full((n, len(ranges), 3), -7, dtype=torch.int64, device="cuda")
    targets = torch.full((n, len(ranges), 4), 99, dtype=torch.int8, device="cuda")
    totals = torch.full((len(ranges), 3), -7, dtype=torch.int64, device="cuda")
    det.process_batch_totals(frames, W, H, LL, LAYOUT_YUYV, ranges, n_frames=n, frame_stride=H * LL,
                             sums=sums, targets=targets, totals=totals)
    torch.cuda.synchronize()
    return sums, targets, totals


@pytest.mark.parametrize("n,kind", [(1024, 0), (1024, 1), (1100, 0), (1000, 0), (2048, 1), (257, 1), (40, 0)])
def test_fused_step_equals_separate_kernels(torch_dev, hsv, oracle_mod, n, kind):
    torch = torch_dev
    frames = _frames(torch, hsv, n, kind)
    want = _separate(torch, hsv, frames, n, BENCH_RANGES)
    det = hsv.Detector(hot=hsv.HOT_CHROMA)
    for rep in range(3):  # the last-workgroup counter resets between launches
        got = _fused(torch, hsv, det, frames, n, BENCH_RANGES)
        for g, w, name in zip(got, want, ("sums", "targets", "totals")):
            assert torch.equal(g, w), (name, n, kind, rep)
    assert det.last_hot_kernel() == hsv.HOT_CHROMA
    det.close()
    assert torch.equal(want[2], want[0].sum(0))
    # sampled frames against the oracle (sums and targets)
    host = frames.view(n, H * LL)
    for f in (0, n // 2, n - 1):
        fr = host[f].cpu().numpy()
        s, t = oracle_mod.batch(fr, H * LL, 1, W, H, LL, oracle_mod.LAYOUT_YUYV, BENCH_RANGES)
        assert np.array_equal(want[0][f].cpu().numpy(), s[0]), f
        assert np.array_equal(want[1][f, :, :3].cpu().numpy(), t[0]), f


def test_fused_step_several_groups(torch_dev, hsv):
    """Six ranges: two launches (4 + 2 ranges), each storing its own columns of
    sums / targets / totals and sharing the handle's scratch."""
    torch = torch_dev
    n = 1024
    ranges = BENCH_RANGES + [(20, 60, 10, 100, 10, 100), (150, 250, 30, 90, 40, 100)]
    frames = _frames(torch, hsv, n, 1)
    want = _separate(torch, hsv, frames, n, ranges)
    det = hsv.Detector(hot=hsv.HOT_CHROMA)
    got = _fused(torch, hsv, det, frames, n, ranges)
    det.close()
    for g, w, name in zip(got, want, ("sums", "targets", "totals")):
        assert torch.equal(g, w), name


def test_fused_step_auto_cold_then_warm(torch_dev, hsv):
    """AUTO: the first batch of a new range set lets the device choose (the
    separate-kernel path), later batches take the fused step; same outputs."""
    torch = torch_dev
    n = 1024
    frames = _frames(torch, hsv, n, 0)
    want = _separate(torch, hsv, frames, n, BENCH_RANGES)
    det = hsv.Detector()
    for _ in range(3):
        got = _fused(torch, hsv, det, frames, n, BENCH_RANGES)
        for g, w, name in zip(got, want, ("sums", "targets", "totals")):
            assert torch.equal(g, w), name
    det.close()


def test_fused_step_two_streams(torch_dev, hsv):
    """Calls on two streams share the handle's fused scratch: ordered, not mixed."""
    torch = torch_dev
    n = 1024
    frames = _frames(torch, hsv, n, 1)
    want = _separate(torch, hsv, frames, n, BENCH_RANGES)
    det = hsv.Detector(hot=hsv.HOT_CHROMA)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for k in range(4):
        s = streams[k % 2]
        sums = torch.empty((n, 4, 3), dtype=torch.int64, device="cuda")
        tg = torch.empty((n, 4, 4), dtype=torch.int8, device="cuda")
        tot = torch.empty((4, 3), dtype=torch.int64, device="cuda")
        with torch.cuda.stream(s):
            det.process_batch_totals(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_frames=n,
                                     frame_stride=H * LL, sums=sums, targets=tg, totals=tot, stream=s)
        outs.append((sums, tg, tot))
    torch.cuda.synchronize()
    det.close()
    for got in outs:
        for g, w, name in zip(got, want, ("sums", "targets", "totals")):
            assert torch.equal(g, w), name


@pytest.mark.parametrize("n,reserve", [(1024, 2), (1100, 32), (40, 5)])
def test_fused_step_with_reserved_cus(torch_dev, hsv, n, reserve):
    """trik_hsv_set_reserved_cus (bench.py's --reserve-cus at N > 1): the hot
    grid is sized to leave CUs free for another stream's kernels, so each
    workgroup takes a larger share of the units; the fused step and the
    separate-kernel path give the same outputs as with every CU, and the call
    returns the previous setting and rejects values outside 0..32."""
    torch = torch_dev
    frames = _frames(torch, hsv, n, 0)
    want = _separate(torch, hsv, frames, n, BENCH_RANGES)
    det = hsv.Detector(hot=hsv.HOT_CHROMA)
    assert det.set_reserved_cus(reserve) == 0
    for _ in range(2):
        got = _fused(torch, hsv, det, frames, n, BENCH_RANGES)
        for g, w, name in zip(got, want, ("sums", "targets", "totals")):
            assert torch.equal(g, w), (name, n, reserve)
    sums = torch.zeros((n, 4, 3), dtype=torch.int64, device="cuda")
    det.batch_sums(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, sums, n_frames=n, frame_stride=H * LL)
    torch.cuda.synchronize()
    assert torch.equal(sums, want[0])
    assert det.last_hot_kernel() == hsv.HOT_CHROMA
    for bad in (-1, 33):
        with pytest.raises(ValueError):
            det.set_reserved_cus(bad)
    assert det.set_reserved_cus(0) == reserve
    det.close()
