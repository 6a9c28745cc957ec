"""The ov7670 multi-blob object sensor on the GPU against
the oracle's literal restatement (oracle/trik_oracle.c:trik_oracle_blob_run;
OSEQ:516-602 with BitmapBuilder BMB:107-217 and Clusterizer CLU:85-202):
metapixel bitmap, label map, label count, the 8 largest clusters after
postProcessing, OutArgs target[8] and the preview -- bit-exact, through the
batched API (trik_hsv_blob_batch / _preview) and the XDAIS quartet
(TRIK_VIDTRANSCODE_CV_create_ov7670)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RED = (0, 20, 80, 20, 50, 50)


@pytest.fixture(scope="module")
def hsv():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import trik_hsv

    return trik_hsv


def _frames(oracle_mod, w, h, ll, cases):
    out = []
    for kind, seed, p in cases:
        if kind == "scene":
            out.append(oracle_mod.blob_scene(w, h, ll, seed, noise=p))
        else:
            rng = np.random.default_rng(seed)
            meta = (rng.random((h // 4, w // 4)) < p).astype(np.uint8)
            out.append(oracle_mod.blob_frame(meta, ll, seed=seed))
    return out


def _check(oracle_mod, res, i, fr, w, h, ll, rng_hsv, what):
    ref = oracle_mod.blob_run(fr, w, h, ll, hsv=rng_hsv, preview=False)
    assert ref["rc"] == 0
    assert np.array_equal(res["meta"][i].cpu().numpy(), ref["meta"]), what
    assert np.array_equal(res["labels"][i].cpu().numpy().view(np.uint16), ref["labels"]), what
    assert int(res["n_labels"][i]) == ref["n_labels"], what
    assert np.array_equal(res["top"][i].cpu().numpy(), ref["top"]), what
    assert np.array_equal(res["targets"][i, :, :3].cpu().numpy(), ref["targets"]), what


# (w, h, ll): VGA, 320x240 with a padded line, bw not a multiple of 64 (K = 2),
# a line length that is not a multiple of 4 (byte loads), tiny, wide (K = 32)
GEOMS = [(640, 480, 640), (320, 240, 352), (352, 96, 352), (320, 240, 322), (32, 4, 32), (8192, 8, 8192)]
CASES = [("scene", 1, 0.0), ("scene", 2, 0.03), ("meta", 3, 0.5), ("meta", 4, 0.75), ("meta", 5, 0.1),
         ("meta", 6, 0.0)]


@pytest.mark.parametrize("hot", ["auto", "chroma"])
@pytest.mark.parametrize("geom", GEOMS)
def test_blob_batch_vs_oracle(hsv, oracle_mod, geom, hot):
    """Both bitmap kernels: the stripe-arithmetic one (AUTO at these batch
    sizes) and the chroma-run one (forced; it needs width % 16 and 16-byte
    aligned lines, else the stripe-arithmetic one runs)."""
    import torch

    w, h, ll = geom
    cases = CASES if w * h <= 640 * 480 else CASES[2:4]
    frames = _frames(oracle_mod, w, h, ll, cases)
    dev = torch.from_numpy(np.concatenate(frames)).cuda()
    det = hsv.Detector(hot=hsv.HOT_CHROMA if hot == "chroma" else hsv.HOT_AUTO)
    try:
        res = det.blob_batch(dev, w, h, ll, RED, meta=True, labels=True)
        chroma_ok = hot == "chroma" and w % 16 == 0 and ll % 16 == 0
        assert det.last_hot_kernel() == (hsv.HOT_CHROMA if chroma_ok else hsv.HOT_STRIPE)
        for i, fr in enumerate(frames):
            _check(oracle_mod, res, i, fr, w, h, ll, RED, (geom, cases[i]))
    finally:
        det.close()


def test_blob_batch_auto_chroma_bitmap(hsv, oracle_mod):
    """A batch past TRIK_HSV_CHROMA_MIN_PIXELS: AUTO builds the bitmap on the
    chroma-run tables; scenes and bitmap-driven frames against the oracle,
    for two ranges (the table rebuild when the sticky range changes)."""
    import torch

    w, h, ll = 640, 480, 640
    cases = [("scene", 10 + i, 0.02 * (i % 3)) for i in range(20)] + \
            [("meta", 40 + i, 0.05 + 0.1 * (i % 6)) for i in range(12)]
    frames = _frames(oracle_mod, w, h, ll, cases)
    dev = torch.from_numpy(np.concatenate(frames)).cuda()
    det = hsv.Detector()
    try:
        for rng_hsv in (RED, (120, 40, 50, 50, 60, 40)):
            res = det.blob_batch(dev, w, h, ll, rng_hsv, meta=True, labels=True)
            assert det.last_hot_kernel() == hsv.HOT_CHROMA
            for i, fr in enumerate(frames):
                _check(oracle_mod, res, i, fr, w, h, ll, rng_hsv, (rng_hsv, cases[i]))
    finally:
        det.close()


def test_blob_batch_strided_and_preview(hsv, oracle_mod):
    import torch

    w, h, ll, n = 320, 240, 320, 12
    fb, stride = 2 * h * ll, 2 * h * ll + 1024
    host = np.zeros(n * stride, np.uint8)
    frames = []
    for i in range(n):
        fr = (oracle_mod.blob_scene(w, h, ll, 40 + i, noise=0.004 * (i % 4),
                                    blobs=((0.2 + 0.05 * i, 0.5, 0.1), (0.8, 0.3 + 0.02 * i, 0.07)))
              if i % 3 else
              oracle_mod.blob_frame((np.random.default_rng(i).random((h // 4, w // 4)) < 0.4).astype(np.uint8),
                                    ll, seed=i))
        host[i * stride:i * stride + fb] = fr
        frames.append(fr)
    dev = torch.from_numpy(host).cuda()
    det = hsv.Detector()
    try:
        res = det.blob_batch(dev, w, h, ll, RED, n_frames=n, frame_stride=stride, meta=True, labels=True)
        for ow, oh, oll in ((160, 120, 320), (200, 150, 401)):
            pv = det.blob_preview(dev, w, h, ll, res["meta"], res["top"], out_width=ow, out_height=oh,
                                  out_line_length=oll, n_frames=n, frame_stride=stride).cpu().numpy()
            for i, fr in enumerate(frames):
                ref = oracle_mod.blob_run(fr, w, h, ll, hsv=RED, out_width=ow, out_height=oh, out_line_length=oll)
                assert np.array_equal(pv[i].reshape(-1), ref["preview"]), (i, ow)
        for i, fr in enumerate(frames):
            _check(oracle_mod, res, i, fr, w, h, ll, RED, i)
    finally:
        det.close()


def _blob_sensor(hsv, w, h, ll, ow, oh, oll):
    s = hsv.BlobSensor(hsv._default_params(1, hsv.FORMAT_YUV422P, max(640, w, ow), max(480, h, oh)))
    assert s.set_params(w, h, ll, out_width=ow, out_height=oh, out_line_length=oll) == 0
    return s


@pytest.mark.parametrize("geom", [(640, 480, 640, 320, 240, 640), (320, 240, 352, 200, 150, 401)])
def test_blob_sensor_process_vs_oracle(hsv, oracle_mod, geom):
    """process() frame after frame with the sticky range: set on the first
    frame and on the fourth, kept otherwise (BMB:110-130)."""
    w, h, ll, ow, oh, oll = geom
    s = _blob_sensor(hsv, w, h, ll, ow, oh, oll)
    state = None
    seq = [RED, None, None, (120, 40, 50, 50, 50, 50), None, RED]
    try:
        for k, rng_hsv in enumerate(seq):
            fr = oracle_mod.blob_scene(w, h, ll, 60 + k, noise=0.01 * (k % 3))
            out = np.full(oh * oll + 16, 0xCD, np.uint8)
            rc, oa = s.process(fr, rng_hsv, out_buffer=out)
            assert rc == 0
            ref = oracle_mod.blob_run(fr, w, h, ll, hsv=rng_hsv, state=state, out_width=ow, out_height=oh,
                                      out_line_length=oll)
            state = ref["state"]
            got = [(oa.alg.target[i].x, oa.alg.target[i].y, oa.alg.target[i].size) for i in range(8)]
            assert got == [tuple(t) for t in ref["targets"].tolist()], (geom, k)
            assert np.array_equal(out[: oh * oll], ref["preview"]), (geom, k)
            assert not out[oh * oll:].any()
    finally:
        s.close()


def test_blob_sensor_range_unset(hsv, oracle_mod):
    """Before any setHsvRange the range is all-zero (uninitialised in the reference)."""
    s = _blob_sensor(hsv, 320, 240, 320, 160, 120, 320)
    try:
        fr = oracle_mod.blob_scene(320, 240, 320, 3)
        out = np.zeros(160 * 120 * 2, np.uint8)
        rc, oa = s.process(fr, None, out_buffer=out)
        ref = oracle_mod.blob_run(fr, 320, 240, 320, hsv=None, out_width=160, out_height=120, out_line_length=320)
        assert rc == 0 and np.array_equal(out, ref["preview"])
        assert all(oa.alg.target[i].size == 0 for i in range(8))
    finally:
        s.close()


def test_blob_rejects(hsv):
    import torch

    with pytest.raises(hsv.TrikHsvError):
        hsv.BlobSensor(hsv._default_params(1, hsv.FORMAT_YUV422))
    det = hsv.Detector()
    try:
        dev = torch.zeros(2 * 64 * 128, dtype=torch.uint8, device="cuda")
        b = hsv._batch(dev, 64, 64, 128, hsv.LAYOUT_YUYV)
        alg = hsv._abi.OV7670InArgsAlg(1, *RED, 0)
        t = torch.empty((1, 8, 4), dtype=torch.int8, device="cuda")
        rc = hsv._lib.trik_hsv_blob_batch(det._h, hsv.C.byref(b), hsv.C.byref(alg), hsv.C.c_void_p(t.data_ptr()),
                                          None, None, None, None, None)
        assert rc != 0 and "ov7670" in hsv._abi.last_error()
        big = torch.zeros(2 * 4096 * 4096, dtype=torch.uint8, device="cuda")
        with pytest.raises(hsv.TrikHsvError):
            det.blob_batch(big, 4096, 4096, 4096, RED)
        empty = det.blob_batch(dev, 64, 64, 64, RED, n_frames=0)
        assert empty["targets"].shape == (0, 8, 4)
    finally:
        det.close()


def test_blob_sensor_empty_frame(hsv):
    """0 x 0 input: no bitmap, no clusters; target[] zeroed (OSEQ:563)."""
    s = hsv.BlobSensor(hsv._default_params(1, hsv.FORMAT_YUV422P))
    try:
        assert s.set_params(0, 0, 0, out_width=0, out_height=0, out_line_length=0) == 0
        out = np.full(16, 0xCD, np.uint8)
        rc, oa = s.process(np.zeros(16, np.uint8), RED, out_buffer=out)
        assert rc == 0
        assert all((oa.alg.target[i].x, oa.alg.target[i].y, oa.alg.target[i].size) == (0, 0, 0) for i in range(8))
        assert not out.any()
    finally:
        s.close()


def test_blob_batch_zero_size_frames(hsv):
    import torch

    det = hsv.Detector()
    try:
        dev = torch.zeros(64, dtype=torch.uint8, device="cuda")
        res = det.blob_batch(dev, 0, 0, 0, RED, n_frames=3, frame_stride=0)
        assert not res["targets"].any() and not res["top"].any() and not res["n_labels"].any()
    finally:
        det.close()


def test_blob_batch_large_from_l2(hsv, oracle_mod):
    """A batch of >= 2 x CUs frames: the clusterer reads the bitmap from L2
    instead of staging it in LDS (more frames resident per CU); small frames
    with random bitmaps of several densities, every frame against the oracle."""
    import torch

    w, h, ll, n = 64, 32, 64, 520
    cases = [("meta", 1000 + i, (0.05, 0.3, 0.55, 0.8)[i % 4]) for i in range(n)]
    frames = _frames(oracle_mod, w, h, ll, cases)
    dev = torch.from_numpy(np.concatenate(frames)).cuda()
    det = hsv.Detector()
    try:
        res = det.blob_batch(dev, w, h, ll, RED, meta=True, labels=True)
        for i, fr in enumerate(frames):
            _check(oracle_mod, res, i, fr, w, h, ll, RED, cases[i])
    finally:
        det.close()


def test_blob_stats_clean_across_geometries(hsv, oracle_mod):
    """One handle, batches of changing geometry: the clusterer's statistics
    buffer is not cleared per batch -- it is zeroed when allocated and every
    clusterer wave zeroes the labels it used before it ends -- so each batch
    here runs on what the previous one (another layout, packed or three-int
    statistics) left behind.  1024 x 1024 takes the unpacked statistics
    (size, sum x, sum y do not fit 63 bits together)."""
    import torch

    seq = [((640, 480, 640), [("meta", 71, 0.5), ("meta", 72, 0.75)]),
           ((1024, 1024, 1024), [("meta", 73, 0.5), ("scene", 74, 0.02)]),
           ((320, 240, 352), [("scene", 75, 0.03), ("meta", 76, 0.3)]),
           ((640, 480, 640), [("meta", 77, 0.75), ("meta", 78, 0.1)]),
           ((1024, 1024, 1024), [("meta", 79, 0.3)])]
    det = hsv.Detector()
    try:
        for (w, h, ll), cases in seq:
            frames = _frames(oracle_mod, w, h, ll, cases)
            dev = torch.from_numpy(np.concatenate(frames)).cuda()
            res = det.blob_batch(dev, w, h, ll, RED, meta=True, labels=True)
            for i, fr in enumerate(frames):
                _check(oracle_mod, res, i, fr, w, h, ll, RED, ((w, h), cases[i]))
    finally:
        det.close()
