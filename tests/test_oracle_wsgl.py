"""The oracle (a restatement of WSEQ, the sequential-pass webcam detector)
against a second reference text: WSGL, the single-pass detector
(trik/webcam/object_sensor/include/internal/cv_ball_detector_singlepass.hpp:
111-161 testifyRgbPixel, 181-213 proceedTwoYuyvPixels, 245-346 run),
restated separately in oracle/trik_oracle_wsgl.c.  The two reference files
compute the same detection and centroid by different routes; here they must
agree on every (Y, U, V) triple, for both pixels of a word, and on whole
frames.  CPU only.  This ties the oracle to a second reference text; it does
not pin parity (the reference cannot run here)."""
import numpy as np
import pytest

from gpu_util import BENCH_RANGES

# the GPU parity tests' edge ranges (tests/test_gpu_parity.py), restated here
# so that this CPU module does not import a GPU-marked one
EDGE_RANGES = [
    (0, 359, 0, 100, 0, 100),
    (10, 10, 100, 100, 100, 100),
    (2, 1, 0, 100, 0, 100),
    (359, 0, 20, 100, 20, 100),
    (400, 500, 200, 250, 0, 255),
    (0, 359, 0, 0, 0, 100),
    (0, 359, 0, 100, 0, 10),
    (120, 120, 0, 100, 0, 100),
]
BAND_RANGES = [(0, 30, 50, 60, 0, 100), (0, 359, 30, 40, 0, 100), (0, 359, 0, 100, 20, 40)]


def oracle_detect(oracle_mod, table, r):
    """WSEQ:171-179 over the oracle's (rgb << 32 | hsv) table, vectorised."""
    f, t, e = oracle_mod.pack_range(r)
    hsv = (table & 0xFFFFFFFF).astype(np.uint32)
    m = np.zeros(hsv.shape, np.uint32)
    for n in range(4):
        b = (hsv >> (8 * n)) & 0xFF
        m |= (((b < ((f >> (8 * n)) & 0xFF)) | (b > ((t >> (8 * n)) & 0xFF))).astype(np.uint32)) << n
    return m == e


@pytest.mark.parametrize("r", BENCH_RANGES + EDGE_RANGES + BAND_RANGES)
def test_wsgl_equals_oracle_all_yuv(oracle_mod, table, r):
    want = oracle_detect(oracle_mod, table, r).astype(np.uint8)
    got = oracle_mod.wsgl_table(r)
    assert np.array_equal(got & 1, want), "first pixel of the word"
    assert np.array_equal(got >> 1, want), "second pixel of the word"
    assert 0 < int(want.sum()) or r[4] > 100 or r in EDGE_RANGES  # the sets detect something


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("w,h,ll", [(640, 480, 1280), (320, 240, 704), (32, 4, 64)])
def test_wsgl_frames_equal_oracle(oracle_mod, kind, w, h, ll):
    frames = oracle_mod.synth(3, w, h, ll, oracle_mod.LAYOUT_YUYV, kind, 0x5EED)
    fb = h * ll
    for i in range(3):
        fr = frames[i * fb:(i + 1) * fb]
        for r in BENCH_RANGES + EDGE_RANGES[:4]:
            sums, _ = oracle_mod.frame(fr, w, h, ll, oracle_mod.LAYOUT_YUYV, [r])
            s, tg = oracle_mod.wsgl_run(fr, w, h, ll, r)
            assert s.tolist() == sums[0].tolist()
            assert tg == oracle_mod.targets(sums[0], w, h)


def test_wsgl_run_rejects_short_buffer(oracle_mod):
    fr = np.zeros(640 * 2 * 479, np.uint8)
    with pytest.raises(ValueError):
        oracle_mod.wsgl_run(fr, 640, 480, 1280, BENCH_RANGES[0])
