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


@pytest.mark.parametrize("layout", [LAYOUT_YUYV, LAYOUT_OV7670])
def test_batch_auto_range_large_batch(hsv, oracle_mod, layout):
    """>= 512 frames take the two-pass kernel, fewer the one-pass kernel with
    256 lanes per frame, <= 32 frames the one with 1024
    (operator.hip:launch_auto_range): all three = the oracle, frame by frame."""
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
