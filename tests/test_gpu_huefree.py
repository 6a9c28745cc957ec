"""GPU parity of the stripe kernel's reduced detection forms
(trik_hsv_stripe.hip, detect_mode): range groups whose every range accepts
every hue (H 0..359 -- the S-band sets) are detected by the sat&val table
alone (kDetectSV), and groups that also accept every saturation (V bands, the
webcam line sensor's range) by the value test alone (kDetectV).  Bit-exact
against the oracle (detectHsvPixel, WSEQ:171-179, with the hue lane always
inside) on every (Y,U,V) triple, in both layouts, and on batches; mixed
groups (one range with a hue bound) keep the full kernel and are checked the
same way.
"""
import numpy as np
import pytest

from gpu_util import LAYOUT_OV7670, LAYOUT_YUYV, T0, exhaustive_yuyv_frame, sums_from_mask

pytestmark = pytest.mark.gpu

S_BANDS = [(0, 359, 20, 25, 0, 100), (0, 359, 40, 45, 0, 100),
           (0, 359, 60, 65, 0, 100), (0, 359, 80, 85, 0, 100)]
V_BANDS = [(0, 359, 0, 100, 20, 25), (0, 359, 0, 100, 40, 45),
           (0, 359, 0, 100, 60, 65), (0, 359, 0, 100, 80, 85)]
HUE_FREE_EDGE = [(0, 359, 0, 100, 0, 100),   # everything
                 (0, 359, 0, 0, 0, 100),     # grey only
                 (0, 359, 0, 100, 0, 10),    # dark only
                 (0, 359, 100, 100, 100, 100)]  # one S, V point
V_EDGE = [(0, 359, 0, 100, 0, 0),      # V = 0 only
          (0, 359, 0, 100, 100, 100),  # V = 255 only
          (0, 359, -5, 120, -10, 3),   # clamped arguments
          (0, 359, 0, 100, 99, 120)]
SETS = {"s_bands": S_BANDS, "v_bands": V_BANDS, "edge": HUE_FREE_EDGE, "v_edge": V_EDGE,
        "one_v": [(0, 359, 0, 100, 30, 70)], "two_s": S_BANDS[:2],
        "mixed": [S_BANDS[0], T0, V_BANDS[1]]}
V_ONLY = ("v_bands", "v_edge", "one_v")


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def stripe(torch_dev):
    import trik_hsv

    d = trik_hsv.Detector(hot=trik_hsv.HOT_STRIPE)
    yield d
    d.close()


def _planar(frame, w, h):
    px = frame.reshape(h, w // 2, 4)
    ylum = np.stack([px[..., 0], px[..., 2]], -1).reshape(h, w)
    chroma = np.stack([px[..., 3], px[..., 1]], -1).reshape(h, w)  # even = V, odd = U
    return np.concatenate([ylum.reshape(-1), chroma.reshape(-1)])


@pytest.mark.parametrize("name", list(SETS))
@pytest.mark.parametrize("layout", [LAYOUT_YUYV, LAYOUT_OV7670])
def test_exhaustive_hue_free(torch_dev, stripe, oracle_mod, name, layout):
    """All 2^24 (Y,U,V) triples through the stripe kernel (masks) vs the oracle."""
    import trik_hsv

    torch = torch_dev
    ranges = SETS[name]
    frame, w, h, ll = exhaustive_yuyv_frame()
    if layout == LAYOUT_OV7670:
        frame, ll = _planar(frame, w, h), w
    _, want = oracle_mod.frame(frame, w, h, ll, layout, ranges, want_mask=True)
    dev = torch.from_numpy(np.ascontiguousarray(frame)).cuda()
    masks, sums = stripe.batch_masks(dev, w, h, ll, layout, ranges)
    assert stripe.last_hot_kernel() == trik_hsv.HOT_STRIPE
    got = masks[0].cpu().numpy()
    bad = np.count_nonzero(got != want)
    assert bad == 0, f"{bad} pixels differ; first at {np.argwhere(got != want)[:5].tolist()}"
    assert sums[0].cpu().numpy().tolist() == sums_from_mask(want, len(ranges)).tolist()


@pytest.mark.parametrize("name,w,h,layout,n", [
    ("s_bands", 640, 480, LAYOUT_YUYV, 24),
    ("v_bands", 640, 480, LAYOUT_YUYV, 24),
    ("one_v", 1280, 720, LAYOUT_YUYV, 6),
    ("one_v", 640, 480, LAYOUT_YUYV, 40),                  # AUTO: the value form at a large batch
    ("v_edge", 640, 480, LAYOUT_YUYV, 8),
    ("v_bands", 320, 240, LAYOUT_OV7670, 16),
    ("mixed", 640, 480, LAYOUT_YUYV, 8),
    ("v_edge", 32, 4, LAYOUT_YUYV, 16),                    # minimal frames: partial tiles
    ("s_bands", 8192, 8, LAYOUT_YUYV, 2),                  # the widest rows the stripe kernel takes
    ("v_bands", 96, 12, LAYOUT_OV7670, 5),
])
@pytest.mark.parametrize("kind", [0, 1])
def test_batches_hue_free(torch_dev, oracle_mod, name, w, h, layout, n, kind):
    """Batches through AUTO and the forced stripe kernel vs the threaded oracle."""
    import trik_hsv

    torch = torch_dev
    ranges = SETS[name]
    ll = 2 * w if layout == LAYOUT_YUYV else w
    fb = trik_hsv.frame_bytes(w, h, ll, layout)
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    trik_hsv.synth(dev, w, h, ll, layout, kind, 0x51DE, first_frame=7)
    host = oracle_mod.synth(n, w, h, ll, layout, kind, 0x51DE, first_frame=7)
    want_s, want_t = oracle_mod.batch(host, fb, n, w, h, ll, layout, ranges, n_threads=8)
    for hot in (trik_hsv.HOT_AUTO, trik_hsv.HOT_STRIPE):
        d = trik_hsv.Detector(hot=hot)
        try:
            sums, tg = d.process_batch(dev, w, h, ll, layout, ranges)
            assert np.array_equal(sums.cpu().numpy(), want_s), (hot, name)
            assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t), (hot, name)
            if name in V_ONLY:  # AUTO keeps value-only groups on the stripe kernel at any size
                assert d.last_hot_kernel() == trik_hsv.HOT_STRIPE
        finally:
            d.close()


@pytest.mark.parametrize("name,layout", [("v_bands", LAYOUT_YUYV), ("s_bands", LAYOUT_YUYV),
                                         ("v_edge", LAYOUT_OV7670)])
def test_padded_lines_hue_free(torch_dev, oracle_mod, name, layout):
    """Padded lineLength and a frame stride that is not the frame size."""
    import trik_hsv

    torch = torch_dev
    ranges = SETS[name]
    w, h, n = 320, 64, 6
    ll = (2 * w if layout == LAYOUT_YUYV else w) + 48
    fb = trik_hsv.frame_bytes(w, h, ll, layout)
    stride = fb + 64
    host = oracle_mod.synth(n, w, h, ll, layout, 1, 0x9A7, first_frame=3)
    padded = np.zeros(n * stride, np.uint8)
    for i in range(n):
        padded[i * stride:i * stride + fb] = host[i * fb:(i + 1) * fb]
    want_s, want_t = oracle_mod.batch(host, fb, n, w, h, ll, layout, ranges, n_threads=8)
    dev = torch.from_numpy(padded).cuda()
    d = trik_hsv.Detector(hot=trik_hsv.HOT_STRIPE)
    try:
        sums, tg = d.process_batch(dev, w, h, ll, layout, ranges, n_frames=n, frame_stride=stride)
        assert np.array_equal(sums.cpu().numpy(), want_s)
        assert np.array_equal(tg[:, :, :3].cpu().numpy(), want_t)
    finally:
        d.close()
