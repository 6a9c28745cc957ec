"""GPU parity of the chroma-run hot kernel (trik_hsv_chroma.hip) against the
CPU oracle, bit-exact, through the C ABI with the kernel forced by
Detector.set_hot_kernel(HOT_CHROMA).

The kernel resolves most YUYV words from per-chroma run descriptors; the
pixels inside a chroma's window, and both pixels of exception-code chromas,
go to its exact path (6 % of words at the bench's 4 ranges, 60 % for the
adversarial band sets below).  The cases cover both paths: every (Y,U,V)
triple, uniform and scene batches at the configs' shapes, several range
groups, strided and padded frames, the table rebuild when the range set
changes, and the AUTO selector's exact-path-share guard.
"""
import numpy as np
import pytest

from gpu_util import (BENCH_RANGES, LAYOUT_OV7670, LAYOUT_YUYV, T0, T1,
                      exhaustive_yuyv_frame, sums_from_mask)
from test_gpu_parity import EDGE_RANGES

pytestmark = pytest.mark.gpu

HOT_CHROMA = 2  # trik_hsv.HOT_CHROMA (the package is imported by the fixtures)


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


@pytest.fixture()
def chroma(hsv, detector):
    """The module's detector with the chroma-run kernel forced."""
    prev = detector.set_hot_kernel(hsv.HOT_CHROMA)
    yield detector
    detector.set_hot_kernel(prev)


def _to_dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


@pytest.mark.parametrize("group", ["bench", "edge"])
def test_chroma_exhaustive_all_yuv_triples(torch_dev, detector, oracle_mod, chroma, group):
    """Every (Y,U,V) triple (verification mode writes each pixel's mask, from
    the run descriptor or the exception row) vs the oracle."""
    torch = torch_dev
    ranges = BENCH_RANGES + EDGE_RANGES[:4] if group == "bench" else EDGE_RANGES
    frame, w, h, ll = exhaustive_yuyv_frame()
    _, want = oracle_mod.frame(frame, w, h, ll, LAYOUT_YUYV, ranges, want_mask=True)
    masks, sums = detector.batch_masks(_to_dev(torch, frame), w, h, ll, LAYOUT_YUYV, ranges)
    assert chroma.last_hot_kernel() == HOT_CHROMA
    got = masks[0].cpu().numpy()
    bad = np.count_nonzero(got != want)
    assert bad == 0, f"{bad} pixels differ; first at {np.argwhere(got != want)[:5].tolist()}"
    assert sums[0].cpu().numpy().tolist() == sums_from_mask(want, len(ranges)).tolist()


def test_chroma_exhaustive_ov7670(torch_dev, detector, oracle_mod, chroma):
    torch = torch_dev
    frame, w, h, ll = exhaustive_yuyv_frame()
    px = frame.reshape(h, w // 2, 4)
    ylum = np.stack([px[..., 0], px[..., 2]], -1).reshape(h, w)
    chrom = np.stack([px[..., 3], px[..., 1]], -1).reshape(h, w)  # even = V, odd = U
    planar = np.concatenate([ylum.reshape(-1), chrom.reshape(-1)])
    _, want = oracle_mod.frame(planar, w, h, w, LAYOUT_OV7670, BENCH_RANGES, want_mask=True)
    masks, sums = detector.batch_masks(_to_dev(torch, planar), w, h, w, LAYOUT_OV7670, BENCH_RANGES)
    assert chroma.last_hot_kernel() == HOT_CHROMA
    assert np.array_equal(masks[0].cpu().numpy(), want)
    assert sums[0].cpu().numpy().tolist() == sums_from_mask(want, 4).tolist()


@pytest.mark.parametrize("w,h,layout,kind,ranges,n", [
    (640, 480, LAYOUT_YUYV, 0, BENCH_RANGES, 24),          # C3 shape, uniform (12 % exceptions)
    (640, 480, LAYOUT_YUYV, 1, BENCH_RANGES, 24),          # C3 shape, scene
    (1280, 720, LAYOUT_YUYV, 0, [T0, T1], 8),              # C4 shape, uniform
    (1280, 720, LAYOUT_YUYV, 1, [T0, T1], 8),              # C4 shape, scene
    (320, 240, LAYOUT_OV7670, 0, [T0], 16),                # C1 layout
    (640, 480, LAYOUT_YUYV, 0, [T0], 3),                   # C2 shape
    (640, 480, LAYOUT_YUYV, 0, BENCH_RANGES + EDGE_RANGES, 4),  # 12 ranges = 3 launches
    (8192, 8, LAYOUT_YUYV, 0, BENCH_RANGES, 6),            # widest row, 3 drain rounds per unpack
    (32, 4, LAYOUT_YUYV, 0, BENCH_RANGES, 40),             # minimal frame, 31 rows per step
    (64, 1000, LAYOUT_OV7670, 0, BENCH_RANGES[:3], 3),     # tall: several tiles per frame
])
def test_chroma_batch_vs_oracle(torch_dev, hsv, detector, oracle_mod, chroma, w, h, layout, kind, ranges, n):
    torch = torch_dev
    ll = 2 * w if layout == LAYOUT_YUYV else w
    fb = hsv.frame_bytes(w, h, ll, layout)
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, layout, kind, 0x7A1C, first_frame=100)
    host = oracle_mod.synth(n, w, h, ll, layout, kind, 0x7A1C, first_frame=100)
    assert np.array_equal(dev.cpu().numpy(), host)
    sums, tg = detector.process_batch(dev, w, h, ll, layout, ranges)
    assert detector.last_hot_kernel() == hsv.HOT_CHROMA
    want_s, want_t = oracle_mod.batch(host, fb, n, w, h, ll, layout, ranges, n_threads=8)
    assert np.array_equal(sums.cpu().numpy(), want_s)
    assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t)


def test_chroma_padded_and_strided(torch_dev, hsv, detector, oracle_mod, chroma):
    """lineLength padding and a frame stride past the frame (16-byte aligned:
    the chroma kernel's vector loads); a misaligned base falls back."""
    torch = torch_dev
    for (w, h, ll, lay) in [(64, 8, 160, LAYOUT_YUYV), (96, 12, 112, LAYOUT_OV7670),
                            (640, 480, 1344, LAYOUT_YUYV)]:
        fb = hsv.frame_bytes(w, h, ll, lay)
        stride = (fb + 48 + 15) // 16 * 16
        n = 5
        host = oracle_mod.synth(n, w, h, ll, lay, 0, 42, frame_stride=stride)
        ranges = BENCH_RANGES + EDGE_RANGES[:2]
        sums, tg = detector.process_batch(_to_dev(torch, host), w, h, ll, lay, ranges, n_frames=n,
                                          frame_stride=stride)
        assert detector.last_hot_kernel() == hsv.HOT_CHROMA, (w, h, ll, lay)
        want_s, want_t = oracle_mod.batch(host, stride, n, w, h, ll, lay, ranges)
        assert np.array_equal(sums.cpu().numpy(), want_s), (w, h, ll, lay)
        assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t), (w, h, ll, lay)
    # a misaligned base cannot take the vector loads: the generic kernel runs
    w, h, ll = 64, 8, 160
    host = oracle_mod.synth(2, w, h, ll, LAYOUT_YUYV, 0, 42)
    buf = np.zeros(host.size + 1, np.uint8)
    buf[1:] = host
    sums, _ = detector.process_batch(_to_dev(torch, buf)[1:], w, h, ll, LAYOUT_YUYV, [T0], n_frames=2)
    assert detector.last_hot_kernel() == hsv.HOT_GENERIC
    want_s, _ = oracle_mod.batch(host, h * ll, 2, w, h, ll, LAYOUT_YUYV, [T0])
    assert np.array_equal(sums.cpu().numpy(), want_s)


def test_chroma_range_set_changes(torch_dev, hsv, detector, oracle_mod, chroma):
    """The chroma tables are rebuilt when the range set changes (and reused
    when it comes back)."""
    torch = torch_dev
    w, h, ll, n = 640, 480, 1280, 6
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 7)
    host = dev.cpu().numpy()
    for ranges in (BENCH_RANGES, [EDGE_RANGES[3], T1], BENCH_RANGES, EDGE_RANGES[4:]):
        sums, _ = detector.process_batch(dev, w, h, ll, LAYOUT_YUYV, ranges)
        want, _ = oracle_mod.batch(host, h * ll, n, w, h, ll, LAYOUT_YUYV, ranges, n_threads=8)
        assert np.array_equal(sums.cpu().numpy(), want), ranges


def test_chroma_equals_stripe_on_full_c3(torch_dev, hsv, oracle_mod):
    """The bench workload (4096 x 640x480, T=4): AUTO picks the chroma kernel,
    its sums and targets equal the stripe kernel's for every frame, and 512 of
    its frames (the first and the last 256) equal the oracle."""
    torch = torch_dev
    w, h, ll, n = 640, 480, 1280, 4096
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C)
    d = hsv.Detector()
    try:
        s_auto, t_auto = d.process_batch(dev, w, h, ll, LAYOUT_YUYV, BENCH_RANGES)
        assert d.last_hot_kernel() == hsv.HOT_CHROMA
        d.set_hot_kernel(hsv.HOT_STRIPE)
        s_str, t_str = d.process_batch(dev, w, h, ll, LAYOUT_YUYV, BENCH_RANGES)
        assert d.last_hot_kernel() == hsv.HOT_STRIPE
    finally:
        d.close()
    assert torch.equal(s_auto, s_str) and torch.equal(t_auto, t_str)
    s, t = s_auto.cpu().numpy(), t_auto.cpu().numpy()
    for first in (0, n - 256):
        host = oracle_mod.synth(256, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C, first_frame=first)
        want_s, want_t = oracle_mod.batch(host, h * ll, 256, w, h, ll, LAYOUT_YUYV, BENCH_RANGES, n_threads=16)
        assert np.array_equal(s[first:first + 256], want_s), first
        assert np.array_equal(t[first:first + 256, :, :3], want_t), first


def test_auto_keeps_small_batches_on_stripe(torch_dev, hsv):
    torch = torch_dev
    dev = torch.zeros(4 * 480 * 1280, dtype=torch.uint8, device="cuda")
    d = hsv.Detector()
    try:
        d.process_batch(dev, 640, 480, 1280, LAYOUT_YUYV, [T0])
        assert d.last_hot_kernel() == hsv.HOT_STRIPE
    finally:
        d.close()


# range sets whose profiles have several separate runs per chroma: most words
# reach the exact path (scripts/adversarial_ranges.py)
S_BANDS = [(0, 359, 20, 25, 0, 100), (0, 359, 40, 45, 0, 100), (0, 359, 60, 65, 0, 100), (0, 359, 80, 85, 0, 100)]
V_BANDS = [(0, 359, 0, 100, 20, 25), (0, 359, 0, 100, 40, 45), (0, 359, 0, 100, 60, 65), (0, 359, 0, 100, 80, 85)]


@pytest.mark.parametrize("ranges", [S_BANDS, V_BANDS], ids=["s_bands", "v_bands"])
def test_chroma_exhaustive_adversarial(torch_dev, detector, oracle_mod, chroma, ranges):
    """Every (Y,U,V) triple through a range set that sends most words to the
    exact path (many windows and exception-code chromas)."""
    torch = torch_dev
    frame, w, h, ll = exhaustive_yuyv_frame()
    _, want = oracle_mod.frame(frame, w, h, ll, LAYOUT_YUYV, ranges, want_mask=True)
    masks, sums = detector.batch_masks(_to_dev(torch, frame), w, h, ll, LAYOUT_YUYV, ranges)
    assert chroma.last_hot_kernel() == HOT_CHROMA
    assert detector.chroma_flagged_share() > 0.5
    got = masks[0].cpu().numpy()
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} pixels differ"
    assert sums[0].cpu().numpy().tolist() == sums_from_mask(want, len(ranges)).tolist()


# hue-bounded S/V bands (scripts/adversarial_ranges.py "hue0-30 S50-60" and
# mixed sets): most chromas stay runs or windows, the share stays low
HUE_BANDS = [(0, 30, 50, 60, 0, 100), (60, 120, 30, 60, 0, 100), (200, 260, 30, 40, 20, 100),
             (330, 20, 50, 60, 30, 100)]


@pytest.mark.parametrize("ranges", [HUE_BANDS[:1], HUE_BANDS], ids=["hue0_30_s50_60", "hue_bands4"])
def test_chroma_exhaustive_hue_bands(torch_dev, detector, oracle_mod, chroma, ranges):
    """Every (Y,U,V) triple through hue-bounded S/V band sets on the chroma kernel."""
    torch = torch_dev
    frame, w, h, ll = exhaustive_yuyv_frame()
    _, want = oracle_mod.frame(frame, w, h, ll, LAYOUT_YUYV, ranges, want_mask=True)
    masks, sums = detector.batch_masks(_to_dev(torch, frame), w, h, ll, LAYOUT_YUYV, ranges)
    assert chroma.last_hot_kernel() == HOT_CHROMA
    got = masks[0].cpu().numpy()
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} pixels differ"
    assert sums[0].cpu().numpy().tolist() == sums_from_mask(want, len(ranges)).tolist()


def test_auto_share_guard(torch_dev, hsv, oracle_mod):
    """AUTO runs the chroma kernel for the bench ranges (share ~2.9 %) and the
    stripe kernel for a range set whose exact-path share is above
    TRIK_HSV_CHROMA_MAX_SHARE; both equal the oracle."""
    torch = torch_dev
    w, h, ll, n = 640, 480, 1280, 32  # TRIK_HSV_CHROMA_MIN_PIXELS
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C, first_frame=9)
    host = dev.cpu().numpy()
    d = hsv.Detector()
    try:
        assert d.chroma_flagged_share() == -1.0
        for ranges, kernel, lo, hi in ((BENCH_RANGES, hsv.HOT_CHROMA, 0.02, 0.04),
                                       (S_BANDS, hsv.HOT_STRIPE, 0.5, 0.7)):
            sums, _ = d.process_batch(dev, w, h, ll, LAYOUT_YUYV, ranges)
            assert d.last_hot_kernel() == kernel
            assert lo < d.chroma_flagged_share() < hi
            want, _ = oracle_mod.batch(host, h * ll, n, w, h, ll, LAYOUT_YUYV, ranges, n_threads=8)
            assert np.array_equal(sums.cpu().numpy(), want)
    finally:
        d.close()


# (layout, w, h, ll): where the past-the-end loads go.  YUYV spans (k + dy)
# rows + 16 bytes of a tile base, ov7670 a luma plane + k rows: VGA YUYV at the
# row bytes, with padding and with 64 KiB lines (1 MiB: larger than the
# ChromaTables block the round-5 kernel read, inside the 4 MiB sink), YUYV
# lines of 272 KiB (4.25 MiB: past the sink, so the tile's last rows are
# re-read), ov7670 VGA (317 KB), ov7670 1280x720 (0.93 MB, larger than the
# ChromaTables block: the geometry that faulted in round 5 would have been
# of this kind), and ov7670 with 9 KiB lines (a 4.4 MB plane: re-read).
TAIL_GEOMS = [
    (LAYOUT_YUYV, 640, 480, 1280),
    (LAYOUT_YUYV, 640, 480, 1296),
    (LAYOUT_YUYV, 640, 480, 65536),
    (LAYOUT_YUYV, 640, 480, 278528),
    (LAYOUT_OV7670, 640, 480, 640),
    (LAYOUT_OV7670, 1280, 720, 1280),
    (LAYOUT_OV7670, 640, 480, 9216),
]


@pytest.mark.parametrize("layout,w,h,ll", TAIL_GEOMS)
def test_chroma_tail_loads_either_side_of_the_sink(torch_dev, hsv, detector, oracle_mod, chroma, layout, w, h, ll):
    """The unconditional load past a tile's last step reads the handle's
    tail sink (KernelArgs::tail, 4 MiB) when every lane's two loads fit inside
    it (chroma_tail_span), else the tile's last rows again: no load depends on
    the address of another allocation.  Geometries on both sides of the sink
    in both layouts (TAIL_GEOMS); the separate-kernel path and the fused step,
    against the oracle."""
    torch = torch_dev
    n = 3
    fb = oracle_mod.frame_bytes(w, h, ll, layout)
    host = oracle_mod.synth(n, w, h, ll, layout, 0, 0x7A1C, first_frame=7)
    dev = _to_dev(torch, host)
    want_s, want_t = oracle_mod.batch(host, fb, n, w, h, ll, layout, BENCH_RANGES, n_threads=8)
    sums, tg = detector.process_batch(dev, w, h, ll, layout, BENCH_RANGES)
    assert detector.last_hot_kernel() == hsv.HOT_CHROMA
    assert np.array_equal(sums.cpu().numpy(), want_s), ll
    assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t), ll
    s2, t2, tot = detector.process_batch_totals(dev, w, h, ll, layout, BENCH_RANGES)
    torch.cuda.synchronize()
    assert np.array_equal(s2.cpu().numpy(), want_s), ll
    assert np.array_equal(t2[:, :, :3].cpu().numpy(), want_t), ll
    assert np.array_equal(tot.cpu().numpy(), want_s.sum(0)), ll
