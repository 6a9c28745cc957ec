"""The webcam line sensor on the GPU (the fourth codec) against
the oracle's restatement of its LineDetector::run (oracle/trik_oracle.c:
trik_oracle_wline_run; LSEQW = trik/webcam/line_sensor/include/internal/
cv_line_detector_seqpass.hpp): OutArgs and the RGB565X preview, bit-exact,
through the XDAIS quartet (TRIK_VIDTRANSCODE_CV_create_webcam_line) and the
exported function table.  The oracle is pinned through its shared parts (the
per-pixel HSV and the range test, checked against the golden vectors); the
line sensor's own composition has no reference fixture ("parity unpinned" for
the overlay and OutArgs arithmetic beyond the restatement)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hsv():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import trik_hsv

    return trik_hsv


def _targets(oa):
    return (oa["target_x"], oa["target_y"], oa["target_size"])


# (w, h, ll, ow, oh, oll): the glue's default portrait output, 2:1 with the
# rows2 preview, a non-dyadic scale with a padded output line, a padded input
# line, same size, tiny
GEOMS = [
    (640, 480, 1280, 240, 320, 480),
    (640, 480, 1280, 320, 240, 640),
    (320, 240, 640, 200, 150, 401),
    (320, 240, 704, 160, 120, 320),
    (320, 240, 640, 320, 240, 640),
    (64, 8, 128, 32, 4, 64),
]
SCENES = [(1, None, 0.25, 0, 30), (2, 30, -0.5, 0, 30), (3, 40, 0.0, 50, 100), (4, None, 0.0, 80, 20),
          (5, 2, 0.0, 0, 100), (6, 300, 0.1, 0, 12)]


def _sensor(hsv, w, h, ll, ow, oh, oll):
    s = hsv.WebcamLineSensor(hsv._default_params(1, hsv.FORMAT_YUV422, max(640, w, ow), max(480, h, oh)))
    assert s.set_params(w, h, ll, out_width=ow, out_height=oh, out_line_length=oll) == 0
    return s


@pytest.mark.parametrize("geom", GEOMS)
def test_webcam_line_process_vs_oracle(hsv, oracle_mod, geom):
    """process() frame after frame: OutArgs (targetY 0) + preview; detect*
    untouched (autoDetectHsv ignored); bytes past the preview cleared."""
    w, h, ll, ow, oh, oll = geom
    s = _sensor(hsv, w, h, ll, ow, oh, oll)
    try:
        for seed, x0, sl, vf, vt in SCENES:
            fr = oracle_mod.wline_scene(w, h, ll, seed, x0=x0 if x0 is None or x0 < w else w // 3, slope=sl)
            out = np.full(oh * oll + 16, 0xCD, np.uint8)
            rc, oa = s.process(fr, (0, 359, 0, 100, vf, vt), out_buffer=out, auto_detect=True)
            assert rc == 0, hsv._abi.last_error()
            rrc, ref, ref_pv, _ = oracle_mod.wline_run(fr, w, h, ll, vf, vt, out_width=ow, out_height=oh,
                                                       out_line_length=oll)
            assert rrc == 0
            assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == _targets(ref), (geom, seed)
            assert (oa.alg.detectHue, oa.alg.detectVal) == (0, 0)
            assert np.array_equal(out[: oh * oll], ref_pv), (geom, seed)
            assert not out[oh * oll:].any()
    finally:
        s.close()


@pytest.mark.parametrize("geom", [(640, 480, 1280, 320, 240, 640), (320, 240, 640, 160, 120, 320),
                                  (320, 240, 640, 200, 150, 401)])
def test_webcam_line_target_at_the_edges(hsv, oracle_mod, geom):
    """A one-pixel line in the first or the last column: the target line's
    columns cx - 1 .. cx + 1 are clamped to the frame (drawOutputPixelBound),
    in the 2:1 pass that draws the overlay itself and in the separate one."""
    w, h, ll, ow, oh, oll = geom
    s = _sensor(hsv, w, h, ll, ow, oh, oll)
    try:
        for seed, x0 in ((11, 0), (12, w - 1), (13, 1), (14, w - 2)):
            fr = oracle_mod.wline_scene(w, h, ll, seed, x0=x0, slope=0.0, line_w=1)
            out = np.full(oh * oll, 0xCD, np.uint8)
            rc, oa = s.process(fr, (0, 359, 0, 100, 0, 30), out_buffer=out)
            assert rc == 0, hsv._abi.last_error()
            rrc, ref, ref_pv, _ = oracle_mod.wline_run(fr, w, h, ll, 0, 30, out_width=ow, out_height=oh,
                                                       out_line_length=oll)
            assert rrc == 0 and abs(ref["target_x"]) >= 98  # the target at an edge
            assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == _targets(ref), (geom, x0)
            assert np.array_equal(out, ref_pv), (geom, x0)
    finally:
        s.close()


def test_webcam_line_hue_and_sat_ignored(hsv, oracle_mod):
    """Only detectValFrom/To are read (LSEQW:345-351): any H/S in InArgs gives
    the same result."""
    w, h, ll = 320, 240, 640
    s = _sensor(hsv, w, h, ll, 160, 120, 320)
    try:
        fr = oracle_mod.wline_scene(w, h, ll, 11)
        outs = []
        for hs in ((0, 359, 0, 100), (10, 20, 90, 95), (300, 40, 0, 0)):
            out = np.zeros(120 * 320, np.uint8)
            rc, oa = s.process(fr, hs + (0, 30), out_buffer=out)
            assert rc == 0, hsv._abi.last_error()
            outs.append(((oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize), out))
        assert all(o[0] == outs[0][0] and np.array_equal(o[1], outs[0][1]) for o in outs)
    finally:
        s.close()


def test_webcam_line_default_params(hsv, oracle_mod):
    """create_webcam_line(NULL): YUV422 in, RGB565X 240x320 preview.  The
    ov7670 YUV422P layout is refused (the glue instantiates YUV422 only).
    (The function table is checked in test_abi_cpu.py / test_xdais_gpu.)"""
    s = hsv.WebcamLineSensor()
    try:
        assert s.set_params(640, 480, 1280, out_width=240, out_height=320, out_line_length=480) == 0
        fr = oracle_mod.wline_scene(640, 480, 1280, 9)
        out = np.zeros(320 * 480, np.uint8)
        rc, oa = s.process(fr, (0, 0, 0, 0, 0, 30), out_buffer=out)
        _, ref, ref_pv, _ = oracle_mod.wline_run(fr, 640, 480, 1280, 0, 30)
        assert rc == 0 and (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == _targets(ref)
        assert ref["target_size"] > 0 and np.array_equal(out, ref_pv)
    finally:
        s.close()
    with pytest.raises(hsv.TrikHsvError):
        hsv.WebcamLineSensor(hsv._default_params(1, hsv.FORMAT_YUV422P))


def test_webcam_line_rejects_and_empty(hsv):
    s = _sensor(hsv, 64, 8, 128, 32, 4, 64)
    try:
        rc, _ = s.process(np.zeros(64 * 8, np.uint8), (0, 359, 0, 100, 0, 30))  # half the frame
        assert rc != 0
    finally:
        s.close()
    s = hsv.WebcamLineSensor()
    try:
        assert s.set_params(0, 0, 0, out_width=0, out_height=0, out_line_length=0) == 0
        out = np.full(16, 0xCD, np.uint8)
        rc, oa = s.process(np.zeros(16, np.uint8), (0, 359, 0, 100, 0, 30), out_buffer=out)
        assert rc == 0 and (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == (0, 0, 0)
        assert not out.any()
    finally:
        s.close()
