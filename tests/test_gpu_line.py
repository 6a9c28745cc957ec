"""The ov7670 line sensor on the GPU against the oracle's
restatement of LineDetector::run (oracle/trik_oracle.c:trik_oracle_line_run;
LSEQ = trik/ov7670/line_sensor/include/internal/cv_line_detector_seqpass.hpp):
per-frame {points, sumX, cross points}, OutArgs and the RGB565X preview,
bit-exact, through the XDAIS quartet (TRIK_VIDTRANSCODE_CV_create_line) and
the batched API (trik_hsv_line_batch / trik_hsv_line_preview)."""
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


# (w, h, ll, ow, oh, oll): the line glue's default portrait output, 2:1, a
# non-dyadic scale with a padded output line, a padded input line, tiny
GEOMS = [
    (640, 480, 640, 240, 320, 480),
    (640, 480, 704, 320, 240, 640),
    (320, 240, 320, 200, 150, 401),
    (320, 240, 384, 160, 120, 320),
    (64, 8, 64, 32, 4, 64),
    (320, 240, 324, 160, 120, 320),  # lineLength % 8 != 0: the generic kernel
]
SCENES = [(1, None, 0.25, 0, 30), (2, 30, -0.5, 0, 30), (3, 40, 0.0, 50, 100), (4, None, 0.0, 80, 20),
          (5, 2, 0.0, 0, 100)]


@pytest.mark.parametrize("geom", GEOMS)
def test_line_batch_and_preview_vs_oracle(hsv, oracle_mod, geom):
    import torch

    w, h, ll, ow, oh, oll = geom
    fb = 2 * h * ll
    frames = [oracle_mod.line_scene(w, h, ll, seed, x0=x0, slope=sl) for seed, x0, sl, _, _ in SCENES]
    dev = torch.from_numpy(np.concatenate(frames)).cuda()
    det = hsv.Detector()
    try:
        for i, (_, _, _, vf, vt) in enumerate(SCENES):
            one = dev[i * fb:(i + 1) * fb]
            for band in (None, (0, h - 1), (h // 3, h // 5)):
                sums, targets = hsv.line_batch(one, w, h, ll, vf, vt, band=band)
                _, oa, _, ref, _ = oracle_mod.line_run(frames[i], w, h, ll, vf, vt, band=band, preview=False)
                assert sums[0].cpu().tolist() == ref.tolist(), (geom, i, band)
                assert tuple(targets[0, :3].cpu().tolist()) == _targets(oa), (geom, i, band)
            sums, _ = hsv.line_batch(one, w, h, ll, vf, vt)
            pv = det.line_preview(one, w, h, ll, vf, vt, sums, out_width=ow, out_height=oh,
                                  out_line_length=oll)
            _, _, ref_pv, _, _ = oracle_mod.line_run(frames[i], w, h, ll, vf, vt, out_width=ow,
                                                     out_height=oh, out_line_length=oll)
            assert np.array_equal(pv[0].cpu().numpy().reshape(-1), ref_pv), (geom, i)
    finally:
        det.close()


def test_line_batch_many_frames(hsv, oracle_mod):
    """Whole-batch launch over N frames (strided) = per-frame oracle runs."""
    import torch

    w, h, ll, n = 320, 240, 352, 24
    fb, stride = 2 * h * ll, 2 * h * ll + 4096
    host = np.zeros(n * stride, np.uint8)
    scenes = []
    for i in range(n):
        fr = oracle_mod.line_scene(w, h, ll, 100 + i, x0=20 + 11 * i, slope=0.1 * (i % 7) - 0.3)
        host[i * stride:i * stride + fb] = fr
        scenes.append(fr)
    dev = torch.from_numpy(host).cuda()
    sums, targets = hsv.line_batch(dev, w, h, ll, 0, 30, n_frames=n, frame_stride=stride)
    det = hsv.Detector()
    try:
        pv = det.line_preview(dev, w, h, ll, 0, 30, sums, n_frames=n, frame_stride=stride)
    finally:
        det.close()
    sums, targets, pv = sums.cpu(), targets.cpu(), pv.cpu().numpy()
    for i, fr in enumerate(scenes):
        _, oa, ref_pv, ref, _ = oracle_mod.line_run(fr, w, h, ll, 0, 30)
        assert sums[i].tolist() == ref.tolist(), i
        assert tuple(targets[i, :3].tolist()) == _targets(oa), i
        assert np.array_equal(pv[i].reshape(-1), ref_pv), i


def _exhaustive_ov7670():
    """A 4096x4096 ov7670 frame holding every (Y, U, V) triple once: pair p
    (2048 per row) has U = p & 255, V = (p >> 8) & 255, Y = 2k, 2k+1 (k = p >> 16)."""
    p = np.arange(1 << 23, dtype=np.int64)
    u, v, k = p & 255, (p >> 8) & 255, p >> 16
    y = np.stack([2 * k, 2 * k + 1], -1).reshape(4096, 4096).astype(np.uint8)
    c = np.stack([v, u], -1).reshape(4096, 4096).astype(np.uint8)
    return np.concatenate([y.reshape(-1), c.reshape(-1)]), y, c


def test_line_exhaustive_v_levels(hsv, table):
    """Every (Y,U,V) triple through the 16-bit V arithmetic: for each percent
    level p, detections with V range [p, p] (and wide ranges) = the per-pixel
    table's counts, sums of columns and band counts."""
    import torch

    fr, y, c = _exhaustive_ov7670()
    W = H = 4096
    Y = y.astype(np.int64)
    V = np.repeat(c[:, 0::2], 2, axis=1).astype(np.int64)
    U = np.repeat(c[:, 1::2], 2, axis=1).astype(np.int64)
    val = (table[Y | (U << 8) | (V << 16)] & 0xFFFFFFFF) >> 16
    cols = np.arange(W)
    win = (cols >= 5) & (cols <= W - 5)
    band = (1000, 1700)
    rows = np.arange(H)
    in_band = (rows >= band[0]) & (rows <= band[1])
    dev = torch.from_numpy(fr).cuda()
    levels = sorted(set(range(0, 101, 1)))
    ranges = [(p, p) for p in levels] + [(0, 30), (31, 100), (0, 100), (50, 99), (1, 100)]
    for vf, vt in ranges:
        lo, hi = (vf * 255) // 100, (vt * 255) // 100
        det = (val >= lo) & (val <= hi) & win[None, :]
        ref = [int(det.sum()), int((det * cols[None, :]).sum()), int(det[in_band].sum())]
        sums, _ = hsv.line_batch(dev, W, H, W, vf, vt, band=band)
        assert sums[0].cpu().tolist() == ref, (vf, vt)


def test_line_wide_frame(hsv, oracle_mod):
    """W > 8192 (column chunks), H = 8 (one row segment)."""
    import torch

    w, h, ll = 8448, 8, 8448
    fr = oracle_mod.line_scene(w, h, ll, 77, x0=6000, slope=1.0, line_w=300)
    dev = torch.from_numpy(fr).cuda()
    for band in (None, (2, 5)):
        sums, targets = hsv.line_batch(dev, w, h, ll, 0, 30, band=band)
        _, oa, _, ref, _ = oracle_mod.line_run(fr, w, h, ll, 0, 30, band=band, preview=False)
        assert sums[0].cpu().tolist() == ref.tolist()
        assert tuple(targets[0, :3].cpu().tolist()) == _targets(oa)


def _line_sensor(hsv, w, h, ll, ow, oh, oll):
    s = hsv.LineSensor(hsv._default_params(1, hsv.FORMAT_YUV422P, max(640, w, ow), max(480, h, oh)))
    assert s.set_params(w, h, ll, out_width=ow, out_height=oh, out_line_length=oll) == 0
    return s


@pytest.mark.parametrize("geom", GEOMS[:4] + GEOMS[5:])
def test_line_sensor_process_vs_oracle(hsv, oracle_mod, geom):
    """process() frame after frame: OutArgs + preview, the cross band carried
    from run to run (LSEQ:298-299, 449-450); detect* untouched (autoDetectHsv
    ignored); bytes past the preview left as process() cleared them."""
    w, h, ll, ow, oh, oll = geom
    s = _line_sensor(hsv, w, h, ll, ow, oh, oll)
    band = None
    try:
        for seed, x0, sl, vf, vt in SCENES:
            fr = oracle_mod.line_scene(w, h, ll, seed, x0=x0, slope=sl)
            out = np.full(oh * oll + 16, 0xCD, np.uint8)
            rc, oa = s.process(fr, (0, 359, 0, 100, vf, vt), out_buffer=out, auto_detect=True)
            assert rc == 0
            _, ref, ref_pv, _, band = oracle_mod.line_run(fr, w, h, ll, vf, vt, band=band, out_width=ow,
                                                          out_height=oh, out_line_length=oll)
            assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == _targets(ref), (geom, seed)
            assert (oa.alg.detectHue, oa.alg.detectVal) == (0, 0)
            assert np.array_equal(out[: oh * oll], ref_pv), (geom, seed)
            assert not out[oh * oll:].any()
    finally:
        s.close()


def test_line_sensor_default_params(hsv, oracle_mod):
    """create_line(NULL): YUV422P in, RGB565X 240x320 preview; 640x480 input."""
    s = hsv.LineSensor()
    try:
        assert s.set_params(640, 480, 640, out_width=240, out_height=320, out_line_length=480) == 0
        fr = oracle_mod.line_scene(640, 480, 640, 9)
        out = np.zeros(320 * 480, np.uint8)
        rc, oa = s.process(fr, (0, 0, 0, 0, 0, 30), out_buffer=out)
        _, ref, ref_pv, _, _ = oracle_mod.line_run(fr, 640, 480, 640, 0, 30, out_width=240, out_height=320,
                                                   out_line_length=480)
        assert rc == 0 and (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == _targets(ref)
        assert np.array_equal(out, ref_pv)
    finally:
        s.close()


def test_line_rejects(hsv, oracle_mod):
    import torch

    # the line sensor takes YUV422P only: YUV422 (packed) create/setup fails
    with pytest.raises(hsv.TrikHsvError):
        hsv.LineSensor(hsv._default_params(1, hsv.FORMAT_YUV422))
    dev = torch.zeros(2 * 64 * 128, dtype=torch.uint8, device="cuda")
    b = hsv._batch(dev, 64, 64, 128, hsv.LAYOUT_YUYV)
    rc = hsv._lib.trik_hsv_line_batch(hsv.C.byref(b), 0, 30, 32, 112, None, None, None)
    assert rc != 0 and "ov7670" in hsv._abi.last_error()
    # input buffer holding only the Y plane (the reference reads both planes)
    s = _line_sensor(hsv, 64, 8, 64, 32, 4, 64)
    try:
        rc, _ = s.process(np.zeros(64 * 8, np.uint8), (0, 359, 0, 100, 0, 30))
        assert rc != 0
        sums, targets = hsv.line_batch(dev, 64, 8, 64, 0, 30, n_frames=0)
        assert sums.shape == (0, 3) and targets.shape == (0, 4)
    finally:
        s.close()


def test_line_sensor_empty_frame(hsv):
    """0 x 0 input: run() skips the image (LSEQ:420); targets 0, preview untouched zeros."""
    s = hsv.LineSensor(hsv._default_params(1, hsv.FORMAT_YUV422P))
    try:
        assert s.set_params(0, 0, 0, out_width=0, out_height=0, out_line_length=0) == 0
        out = np.full(16, 0xCD, np.uint8)
        rc, oa = s.process(np.zeros(16, np.uint8), (0, 359, 0, 100, 0, 30), out_buffer=out)
        assert rc == 0 and (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == (0, 0, 0)
        assert not out.any()
    finally:
        s.close()
