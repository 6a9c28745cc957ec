"""The operator's other outputs on the GPU against the
oracle's restatement of BallDetector::run (oracle/trik_oracle.c:trik_oracle_run):

* the RGB565X preview stream -- proceedImageHsv's per-pixel writes through
  the truncated scale maps plus the guide lines and target circle
  (WSEQ:66-166, 316-354, 371-387, 471-494);
* autoDetectHsv -- HsvRangeDetector::detect (trik/webcam/object_sensor/
  include/internal/cv_hsv_range_detector.hpp:88-198).

Byte-exact, through both the XDAIS process() call and the batched API."""
import numpy as np
import pytest

from gpu_util import LAYOUT_OV7670, LAYOUT_YUYV, T0, T1, T3

pytestmark = pytest.mark.gpu

SEED = 0x7A1C
FULL = (0, 359, 0, 100, 0, 100)


@pytest.fixture(scope="module")
def hsv():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import trik_hsv

    return trik_hsv


def _sensor(hsv, w, h, ll, ow, oh, oll, layout):
    fmt = hsv.FORMAT_YUV422 if layout == LAYOUT_YUYV else hsv.FORMAT_YUV422P
    # create() runs setup with the default 640x480 dynamic params (WGLUE:205-266)
    s = hsv.ObjectSensor(hsv._default_params(1, fmt, max(640, w, ow), max(480, h, oh)))
    assert s.set_params(w, h, ll, out_width=ow, out_height=oh, out_line_length=oll) == 0
    return s


# (w, h, ll, ow, oh, oll, layout): 2:1 (the reference default), identity, a
# non-dyadic scale (0.625), a padded output line, a width-bound scale, ov7670
GEOMS = [
    (640, 480, 1280, 320, 240, 640, LAYOUT_YUYV),
    (320, 240, 640, 320, 240, 640, LAYOUT_YUYV),
    (320, 240, 640, 200, 150, 400, LAYOUT_YUYV),
    (320, 240, 704, 160, 120, 333, LAYOUT_YUYV),
    (256, 240, 512, 100, 200, 200, LAYOUT_YUYV),
    (320, 240, 320, 160, 120, 320, LAYOUT_OV7670),
    # upscaled (output pixels nobody writes: -1 in the maps), and maps too
    # large for the gather kernel's LDS (out_w + out_h > 1536: read from memory)
    (160, 120, 320, 320, 240, 640, LAYOUT_YUYV),
    (1024, 768, 2048, 1024, 768, 2048, LAYOUT_YUYV),
]


@pytest.mark.parametrize("geom", GEOMS)
@pytest.mark.parametrize("kind,rng,auto", [(1, T0, True), (0, T3, True), (1, FULL, False)])
def test_process_preview_and_auto_range(hsv, oracle_mod, geom, kind, rng, auto):
    w, h, ll, ow, oh, oll, layout = geom
    s = _sensor(hsv, w, h, ll, ow, oh, oll, layout)
    frame = oracle_mod.synth(1, w, h, ll, layout, kind, SEED, first_frame=3)
    out = np.full(oh * oll + 16, 0xCD, np.uint8)
    rc, oa = s.process(frame, rng, out_buffer=out, auto_detect=auto)
    assert rc == 0
    rc_o, want, preview = oracle_mod.run(frame, w, h, ll, layout, rng, auto_detect=auto,
                                         out_width=ow, out_height=oh, out_line_length=oll)
    assert rc_o == 0
    assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == (
        want["target_x"], want["target_y"], want["target_size"])
    bad = np.flatnonzero(out[:oh * oll] != preview)
    assert bad.size == 0, f"{bad.size} preview bytes differ, first at {bad[:6].tolist()}"
    assert not out[oh * oll:].any()
    got_detect = (oa.alg.detectHue, oa.alg.detectHueTolerance, oa.alg.detectSat,
                  oa.alg.detectSatTolerance, oa.alg.detectVal, oa.alg.detectValTolerance)
    if auto:
        assert got_detect == (want["detect_hue"], want["detect_hue_tol"], want["detect_sat"],
                              want["detect_sat_tol"], want["detect_val"], want["detect_val_tol"])
    else:
        assert got_detect == (0, 0, 0, 0, 0, 0)  # untouched (WSEQ:455-462)
    s.close()


def test_process_without_target_and_without_preview(hsv, oracle_mod):
    w, h, ll = 320, 240, 640
    frame = oracle_mod.synth(1, w, h, ll, LAYOUT_YUYV, 1, SEED)
    empty = (10, 10, 100, 100, 100, 100)  # nothing matches: lines only, no circle
    s = _sensor(hsv, w, h, ll, 160, 120, 320, LAYOUT_YUYV)
    out = np.zeros(120 * 320, np.uint8)
    rc, oa = s.process(frame, empty, out_buffer=out)
    _, want, preview = oracle_mod.run(frame, w, h, ll, LAYOUT_YUYV, empty, out_width=160,
                                      out_height=120, out_line_length=320)
    assert rc == 0 and oa.alg.targetSize == 0 and np.array_equal(out, preview)
    s.close()
    s0 = hsv.ObjectSensor(hsv._default_params(0))  # numOutputStreams = 0: nothing written
    assert s0.set_params(w, h, ll) == 0
    rc, oa = s0.process(frame, T0, auto_detect=True)
    _, want, _ = oracle_mod.run(frame, w, h, ll, LAYOUT_YUYV, T0, auto_detect=True, preview=False)
    assert rc == 0 and oa.alg.detectHue == want["detect_hue"]
    s0.close()


@pytest.mark.parametrize("w,h,ll,layout,kind", [
    (640, 480, 1280, LAYOUT_YUYV, 0),    # uniform: many histogram ties
    (640, 480, 1280, LAYOUT_YUYV, 1),
    (1280, 720, 2560, LAYOUT_YUYV, 1),   # C4 geometry
    (320, 240, 320, LAYOUT_OV7670, 0),
    (32, 4, 64, LAYOUT_YUYV, 0),         # step = 0: empty zone, all zero
    (32, 480, 64, LAYOUT_YUYV, 1),       # hWidth < step: uint16 wrap of the zone bounds
    (64, 8, 128, LAYOUT_YUYV, 0),        # step = 1: a single... empty zone (strict bounds)
    (96, 24, 192, LAYOUT_YUYV, 0),       # step = 4: 7x7 zone
])
def test_batch_auto_range(hsv, oracle_mod, w, h, ll, layout, kind):
    import torch

    n = 6
    fb = hsv.frame_bytes(w, h, ll, layout)
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, layout, kind, SEED, first_frame=40)
    got = hsv.batch_auto_range(dev, w, h, ll, layout).cpu().numpy().astype(np.int64)
    host = dev.cpu().numpy()
    for f in range(n):
        _, want, _ = oracle_mod.run(host[f * fb:(f + 1) * fb], w, h, ll, layout, T0,
                                    auto_detect=True, preview=False)
        assert got[f].tolist() == [want["detect_hue"], want["detect_hue_tol"], want["detect_sat"],
                                   want["detect_sat_tol"], want["detect_val"],
                                   want["detect_val_tol"]], f


def _auto_want(oracle_mod, host, fb, n, w, h, ll, layout):
    out = []
    for f in range(n):
        _, want, _ = oracle_mod.run(host[f * fb:(f + 1) * fb], w, h, ll, layout, T0,
                                    auto_detect=True, preview=False)
        out.append([want["detect_hue"], want["detect_hue_tol"], want["detect_sat"],
                     want["detect_sat_tol"], want["detect_val"], want["detect_val_tol"]])
    return out


@pytest.mark.parametrize("layout", [LAYOUT_YUYV, LAYOUT_OV7670])
def test_batch_auto_range_large_batch(hsv, oracle_mod, layout):
    """16-byte aligned batches take the chunked two-pass kernel
    (auto_range_vec_kernel) at every batch size: 520, 64 and 16 frames of the
    same data agree with each other and with the oracle, frame by frame.
    (The one-pass fallback kernels: test_batch_auto_range_fallback_kernels.)"""
    import torch

    w, h, n = 160, 120, 520
    ll = 2 * w if layout == LAYOUT_YUYV else w
    fb = hsv.frame_bytes(w, h, ll, layout)
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, layout, 1, SEED + 7, first_frame=3)
    got = hsv.batch_auto_range(dev, w, h, ll, layout).cpu().numpy().astype(np.int64)
    few = hsv.batch_auto_range(dev[:16 * fb], w, h, ll, layout).cpu().numpy().astype(np.int64)
    assert np.array_equal(got[:16], few)
    mid = hsv.batch_auto_range(dev[:64 * fb], w, h, ll, layout).cpu().numpy().astype(np.int64)
    assert np.array_equal(got[:64], mid)
    host = dev.cpu().numpy()
    for f in range(n):
        _, want, _ = oracle_mod.run(host[f * fb:(f + 1) * fb], w, h, ll, layout, T0,
                                    auto_detect=True, preview=False)
        assert got[f].tolist() == [want["detect_hue"], want["detect_hue_tol"], want["detect_sat"],
                                   want["detect_sat_tol"], want["detect_val"],
                                   want["detect_val_tol"]], f


# Batches launch_auto_range cannot give the chunked kernel (a frames pointer
# 4 bytes past a 16-byte boundary, or a line length that is not a multiple of
# 16): <= 32 frames run auto_range_kernel<1024>, more auto_range_kernel<256>.
@pytest.mark.parametrize("w,h,ll,layout,n,offset", [
    (640, 480, 1280, LAYOUT_YUYV, 6, 4),      # misaligned base, <1024>
    (640, 480, 1280, LAYOUT_YUYV, 40, 4),     # misaligned base, <256>
    (96, 72, 200, LAYOUT_YUYV, 8, 0),         # line length % 16 == 8, <1024>
    (96, 72, 200, LAYOUT_YUYV, 48, 0),        # <256>
    (320, 240, 324, LAYOUT_OV7670, 5, 0),     # ov7670, line length % 16 == 4, <1024>
    (320, 240, 320, LAYOUT_OV7670, 36, 4),    # ov7670 misaligned base, <256>
])
def test_batch_auto_range_fallback_kernels(hsv, oracle_mod, w, h, ll, layout, n, offset):
    import torch

    fb = hsv.frame_bytes(w, h, ll, layout)
    raw = torch.empty(n * fb + 16, dtype=torch.uint8, device="cuda")
    dev = raw[offset:offset + n * fb]
    assert dev.data_ptr() % 16 == offset
    hsv.synth(dev, w, h, ll, layout, 1, SEED + 3, first_frame=11)
    got = hsv.batch_auto_range(dev, w, h, ll, layout).cpu().numpy().astype(np.int64)
    host = dev.cpu().numpy()
    assert got.tolist() == _auto_want(oracle_mod, host, fb, n, w, h, ll, layout)


def test_batch_auto_range_single_colour_frames(hsv, table):
    """Every (U, V) at six Y levels, one colour per frame (96x24, a 7x7 zone,
    393,216 frames): each channel's winner is the colour's own H, S and V, so
    the output is (H x 1.4, S x 0.39, V x 0.39) with the reference's float
    constants (hpp:190-195) -- the chunked kernel's packed two-pixel HSV
    (hsv_key2: both pixels of a word in 16-bit halves, the B channel's 16-bit
    wrap) against the oracle's table on every one of those (Y, U, V).  H is
    checked exactly (1.4 H is injective), S and V through the scaling."""
    import torch

    w, h, ll = 96, 24, 192
    ys = [0, 37, 100, 160, 222, 255]
    uv = np.arange(65536, dtype=np.int64)
    U, V = uv & 255, uv >> 8
    Y = np.repeat(np.array(ys, np.int64), 65536)
    U, V = np.tile(U, len(ys)), np.tile(V, len(ys))
    word = Y | (U << 8) | (Y << 16) | (V << 24)
    word = np.where(word >= 1 << 31, word - (1 << 32), word).astype(np.int32)
    n, per = word.size, h * ll // 4
    dev = torch.from_numpy(word).cuda().view(-1, 1).expand(n, per).contiguous().view(torch.uint8).reshape(-1)
    got = hsv.batch_auto_range(dev, w, h, ll, LAYOUT_YUYV).cpu().numpy().astype(np.int64)
    e = table[Y | (U << 8) | (V << 16)] & 0xFFFFFFFF
    H, S, Vv = e & 0xFF, (e >> 8) & 0xFF, (e >> 16) & 0xFF
    k14, k39 = np.float64(np.float32(1.4)), np.float64(np.float32(0.39))
    want = np.stack([(H * k14).astype(np.uint16), np.full(n, 15), (S * k39).astype(np.uint16), np.full(n, 30),
                     (Vv * k39).astype(np.uint16), np.full(n, 30)], 1).astype(np.int64)
    bad = np.flatnonzero((got != want).any(1))
    assert bad.size == 0, [(int(Y[i]), int(U[i]), int(V[i]), got[i].tolist(), want[i].tolist()) for i in bad[:5]]


def _zone_hsv(table, fr, w, h, ll):
    """The strict central zone's per-pixel (H, S, V) of a YUYV frame in scan
    order (cv_hsv_range_detector.hpp:88-108 bounds), from the oracle's table."""
    px = fr[: h * ll].reshape(h, ll)[:, : 2 * w].reshape(h, w // 2, 4).astype(np.int64)
    Y = np.stack([px[..., 0], px[..., 2]], -1).reshape(h, w)
    U = np.repeat(px[..., 1], 2, axis=1)
    V = np.repeat(px[..., 3], 2, axis=1)
    step = h // 6
    r0, r1, c0, c1 = h // 2 - step + 1, h // 2 + step, w // 2 - step + 1, w // 2 + step
    e = table[(Y | (U << 8) | (V << 16))[r0:r1, c0:c1]].reshape(-1) & 0xFFFFFFFF
    return [(e >> sh) & 0xFF for sh in (0, 8, 16)]


def _tie_frame(w, h, ll, first):
    """A YUYV frame whose central zone holds two colours with equal counts
    (54 zone rows each, 8,586 pixels) and a third with fewer (51 rows): every
    channel's maximum count is tied between A = (Y 100, U 90, V 200), HSV
    (7, 230, 211), and B = (Y 60, U 200, V 90), HSV (158, 254, 196); the third
    colour is grey (Y 120), HSV (85, 0, 120).  `first` ('A' or 'B') fills the
    upper 54 zone rows: its last occurrence comes first, so the sequential
    arg-max picks it in every channel."""
    words = np.zeros((h, ll // 4, 4), np.uint8)
    words[:, :, :] = (120, 128, 120, 128)
    A, B = (100, 90, 100, 200), (60, 200, 60, 90)
    step = h // 6
    r0, c0, c1 = h // 2 - step + 1, w // 2 - step + 1, w // 2 + step  # zone rows r0.., columns c0..c1-1
    k0, k1 = c0 // 2, (c1 - 1) // 2 + 1  # words holding zone pixels
    top, bottom = (A, B) if first == "A" else (B, A)
    words[r0:r0 + 54, k0:k1] = top
    words[r0 + 54:r0 + 108, k0:k1] = bottom
    return words.reshape(-1)


def test_batch_auto_range_pass2_ties(hsv, oracle_mod, table):
    """The chunked kernel's second pass (operator.hip: the last occurrences of
    values tied at the maximum count) decides frames where several values
    share a channel's maximum count: the sequential arg-max (strict >) picks
    the value whose last occurrence comes first, which need not be the
    smallest tied value that pass 1 alone would give.  520 VGA frames: every
    4th a constructed tie in all three channels (_tie_frame, A or B first),
    the rest uniform bytes.  The test asserts that the tie frames are ones
    where pass 2 changes the answer, and that every frame equals the oracle."""
    import torch

    w, h, ll, n = 640, 480, 1280, 520
    fb = h * ll
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, SEED + 11, first_frame=0)
    ties = {f: ("A" if f % 8 == 0 else "B") for f in range(0, n, 4)}
    for f, first in ties.items():
        dev[f * fb:(f + 1) * fb] = torch.from_numpy(_tie_frame(w, h, ll, first)).cuda()
    got = hsv.batch_auto_range(dev, w, h, ll, LAYOUT_YUYV).cpu().numpy().astype(np.int64)
    host = dev.cpu().numpy()
    decisive = set()
    for f in ties:
        for ch in _zone_hsv(table, host[f * fb:(f + 1) * fb], w, h, ll):
            cnt = np.bincount(ch, minlength=256)
            tied = np.flatnonzero(cnt == cnt.max())
            assert tied.size == 2, f
            last = {int(v): int(np.flatnonzero(ch == v)[-1]) for v in tied}
            if min(last, key=last.get) != int(tied[0]):
                decisive.add(f)
    assert decisive == set(ties), "every tie frame has a channel where pass 2 changes the answer"
    assert got.tolist() == _auto_want(oracle_mod, host, fb, n, w, h, ll, LAYOUT_YUYV)


@pytest.mark.parametrize("w,h,ll,ow,oh,oll,layout,kind", [
    (640, 480, 1280, 320, 240, 640, LAYOUT_YUYV, 1),
    (640, 480, 1280, 320, 240, 640, LAYOUT_YUYV, 0),
    (320, 240, 640, 200, 150, 401, LAYOUT_YUYV, 1),
    (320, 240, 320, 160, 120, 320, LAYOUT_OV7670, 1),
    # square frames: 2:1 maps whose written columns end before out_w (the row
    # kernel would load past the row; the gather takes them)
    (480, 480, 960, 320, 240, 640, LAYOUT_YUYV, 1),
    (256, 256, 256, 160, 128, 320, LAYOUT_OV7670, 1),
])
def test_batch_preview(hsv, oracle_mod, w, h, ll, ow, oh, oll, layout, kind):
    import torch

    n, ranges = 5, [T0, T1, T3]
    fb = hsv.frame_bytes(w, h, ll, layout)
    dev = torch.empty(n * fb, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, layout, kind, SEED, first_frame=11)
    det = hsv.Detector()
    sums, _ = det.process_batch(dev, w, h, ll, layout, ranges)
    host = dev.cpu().numpy()
    for t, rng in enumerate(ranges):
        pv = det.batch_preview(dev, w, h, ll, layout, rng, sums[:, t:, :], out_width=ow,
                               out_height=oh, out_line_length=oll, sums_pitch=len(ranges))
        pv = pv.cpu().numpy().reshape(n, -1)
        for f in range(n):
            _, _, want = oracle_mod.run(host[f * fb:(f + 1) * fb], w, h, ll, layout, rng,
                                        out_width=ow, out_height=oh, out_line_length=oll)
            assert np.array_equal(pv[f], want), (t, f)
    det.close()
