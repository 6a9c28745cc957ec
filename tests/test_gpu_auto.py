"""AUTO's measured share (trik_hsv_abi.cpp: poll_measured / plan_hot /
probe_measured): input concentrated on the chromas the chroma-run tables
describe worst goes to the stripe kernel after a few batches, although the
range set's expected (uniform-input) share keeps it on the chroma-run kernel;
every batch's sums stay identical to the stripe kernel's (and so to the oracle,
tests/test_gpu_parity.py).

The adversarial frames use chromas U = 245..254, V = 0: for the bench ranges
every one of them is an exception chroma (the B channel's 16-bit wrap at high
Y, WSEQ:195-205, gives profiles T2 / 0 / T1 that no run descriptor holds), so
both pixels of every word go to the exact path.
"""

import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

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


def _exception_frames(torch, n):
    g = torch.Generator(device="cuda").manual_seed(7)
    words = n * H * LL // 4
    y0 = torch.randint(0, 256, (words,), device="cuda", generator=g, dtype=torch.int64)
    y1 = torch.randint(0, 256, (words,), device="cuda", generator=g, dtype=torch.int64)
    u = torch.randint(245, 255, (words,), device="cuda", generator=g, dtype=torch.int64)
    w = (y0 | (u << 8) | (y1 << 16)).to(torch.int32)  # V = 0
    return w.view(torch.uint8)


def test_auto_moves_concentrated_input_to_stripe(torch_dev, hsv):
    torch = torch_dev
    n = 1024
    frames = _exception_frames(torch, n)
    ref = hsv.Detector(hot=hsv.HOT_STRIPE)
    want, _ = ref.process_batch(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES)
    torch.cuda.synchronize()
    ref.close()
    det = hsv.Detector()
    ran = []
    for _ in range(20):
        sums, _ = det.process_batch(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES)
        torch.cuda.synchronize()
        assert torch.equal(sums, want)
        ran.append(det.last_hot_kernel())
    assert det.chroma_flagged_share() < 0.05  # the uniform-input expectation
    assert det.chroma_measured_share() > 0.9  # what these frames give
    assert ran[1] == hsv.HOT_CHROMA, ran
    assert all(k == hsv.HOT_STRIPE for k in ran[-5:]), ran
    det.close()


def test_auto_measures_a_later_group(torch_dev, hsv):
    """A first group of value-only ranges runs the stripe kernel's value form
    under AUTO; the second group (the bench ranges) runs the chroma-run kernel.
    Its measured share must still be read back and move it to the stripe
    kernel on concentrated input (the readback used to count group
    0's chroma-run launches only)."""
    torch = torch_dev
    n = 1024
    frames = _exception_frames(torch, n)
    vbands = [(0, 359, 0, 100, 10 + 20 * i, 20 + 20 * i) for i in range(4)]
    ranges = vbands + list(BENCH_RANGES)
    ref = hsv.Detector(hot=hsv.HOT_STRIPE)
    want, _ = ref.process_batch(frames, W, H, LL, LAYOUT_YUYV, ranges)
    torch.cuda.synchronize()
    ref.close()
    det = hsv.Detector()
    ran = []
    for _ in range(20):
        sums, _ = det.process_batch(frames, W, H, LL, LAYOUT_YUYV, ranges)
        torch.cuda.synchronize()
        assert torch.equal(sums, want)
        ran.append(det.last_hot_kernel())
    assert ran[1] == hsv.HOT_MIXED, ran  # group 0 stripe (value form), group 1 chroma-run
    assert det.chroma_measured_share() > 0.9
    assert all(k == hsv.HOT_STRIPE for k in ran[-5:]), ran
    det.close()


def test_auto_keeps_uniform_input_on_chroma(torch_dev, hsv):
    torch = torch_dev
    n = 1024
    frames = torch.empty(n * H * LL, dtype=torch.uint8, device="cuda")
    hsv.synth(frames, W, H, LL, LAYOUT_YUYV, 0, 0x7A1C)
    det = hsv.Detector()
    for _ in range(12):
        det.process_batch(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES)
        torch.cuda.synchronize()
    assert det.last_hot_kernel() == hsv.HOT_CHROMA
    m = det.chroma_measured_share()
    assert abs(m - det.chroma_flagged_share()) < 0.005, m  # uniform bytes: measured = expected
    det.close()


def test_auto_wide_rows_cold_set_counts_once(torch_dev, hsv, oracle_mod):
    """Rows wider than the stripe kernel takes (9600 px: the chroma kernel's
    wide mode, the stripe kernel's geometry refuses them) with a range set new
    to the handle: the first batch is planned before the set's share is known
    (gated launches); the sums must be counted once, equal to the oracle, on
    the cold batch and the warm one (a gated chroma launch must not
    be followed by an ungated partner)."""
    torch = torch_dev
    w, h, n = 9600, 64, 20  # 20 * 9600 * 64 px >= TRIK_HSV_CHROMA_MIN_PIXELS
    ll = 2 * w
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C)
    want, _ = oracle_mod.batch(dev.cpu().numpy(), h * ll, n, w, h, ll, LAYOUT_YUYV, BENCH_RANGES, n_threads=16)
    d = hsv.Detector()
    try:
        for _ in range(2):  # cold range set, then warm
            sums, _ = d.process_batch(dev, w, h, ll, LAYOUT_YUYV, BENCH_RANGES)
            torch.cuda.synchronize()
            assert (sums.cpu().numpy() == want).all()
    finally:
        d.close()


def test_empty_batch_keeps_gated_answer(torch_dev, hsv):
    """a first batch of a new range set is planned on the device
    (gated launches: the builder's cost is not back yet); an empty batch after
    it must keep that call's answer, and last_hot_kernel() resolve it to a
    valid kind (it returned the negative partner code when the empty call
    dropped the pending set)."""
    torch = torch_dev
    n = 64
    frames = torch.empty(n * H * LL, dtype=torch.uint8, device="cuda")
    hsv.synth(frames, W, H, LL, LAYOUT_YUYV, 0, 0x7A1C)
    det = hsv.Detector()
    det.process_batch(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES)
    det.process_batch(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_frames=0)
    torch.cuda.synchronize()
    assert det.last_hot_kernel() == hsv.HOT_CHROMA
    det.close()
