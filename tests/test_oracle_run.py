"""The oracle's whole-run restatement (trik_oracle_run: preview stream,
overlays, autoDetectHsv, OutArgs) checked three ways on the CPU:

* against the committed golden runs (tests/golden/oracle_golden.json);
* against independent Python restatements built on the per-pixel table:
  - HsvRangeDetector::detect as the reference's literal sequential loop
    (cv_hsv_range_detector.hpp:122-198, running arg-max with strict >);
  - the preview: last-writer scan over truncated double scale maps, then the
    guide lines and the midpoint circle (WSEQ:66-166, 316-354, 371-387,
    471-494);
* for consistency with trik_oracle_frame / trik_oracle_targets.
"""
import hashlib
import math

import numpy as np
import pytest

T0 = (0, 30, 50, 100, 30, 100)
T3 = (330, 20, 30, 100, 30, 100)


def test_golden_runs(oracle_mod, golden):
    for c in golden["runs"]:
        fr = oracle_mod.synth(1, c["width"], c["height"], c["line_length"], c["layout"], c["kind"],
                              c["seed"], first_frame=c["frame"])
        rc, oa, pv = oracle_mod.run(fr, c["width"], c["height"], c["line_length"], c["layout"],
                                    tuple(golden["ranges"][c["range"]]), auto_detect=bool(c["auto"]),
                                    out_width=c["out_width"], out_height=c["out_height"],
                                    out_line_length=c["out_line_length"])
        assert rc == 0
        assert hashlib.sha256(pv.tobytes()).hexdigest() == c["preview_sha256"], c["name"]
        assert oa == c["outargs"], c["name"]


def _hsv_image(oracle_mod, table, fr, w, h, ll, layout):
    """Per-pixel (rgb888, hsv) from the 2^24 table (independent of the frame walk)."""
    if layout == oracle_mod.LAYOUT_YUYV:
        px = fr[: h * ll].reshape(h, ll)[:, : 2 * w].reshape(h, w // 2, 4).astype(np.int64)
        Y = np.stack([px[..., 0], px[..., 2]], -1).reshape(h, w)
        U = np.repeat(px[..., 1], 2, axis=1)
        V = np.repeat(px[..., 3], 2, axis=1)
    else:
        Y = fr[: h * ll].reshape(h, ll)[:, :w].astype(np.int64)
        c = fr[h * ll: 2 * h * ll].reshape(h, ll)[:, :w].astype(np.int64)
        V = np.repeat(c[:, 0::2], 2, axis=1)
        U = np.repeat(c[:, 1::2], 2, axis=1)
    e = table[Y | (U << 8) | (V << 16)]
    return (e >> 32).astype(np.int64), (e & 0xFFFFFFFF).astype(np.int64)


def _auto_range_loop(hsv, w, h):
    """cv_hsv_range_detector.hpp:88-198, literally (uint16 zone bounds)."""
    u16 = lambda v: v & 0xFFFF  # noqa: E731
    hh, hw, step = u16(h // 2), u16(w // 2), u16(h // 6)
    lp, rp, tp, bp = u16(hw - step), u16(hw + step), u16(hh - step), u16(hh + step)
    out = []
    for sh in (0, 8, 16):
        hist = [0] * 256
        best, best_n = 0, 0
        for row in range(h):
            if not (tp < row < bp):
                continue
            for col in range(w):
                if lp < col < rp:
                    x = (int(hsv[row, col]) >> sh) & 255
                    hist[x] += 1
                    if hist[x] > best_n:
                        best, best_n = x, hist[x]
        out.append(best)
    f14, f39 = float(np.float32(1.4)), float(np.float32(0.39))
    return [int(out[0] * f14), 15, int(out[1] * f39), 30, int(out[2] * f39), 30]


@pytest.mark.parametrize("w,h,ll,layout,kind,frame", [
    (64, 48, 128, 0, 0, 1), (64, 48, 128, 0, 1, 2), (96, 96, 192, 0, 0, 3),
    (64, 48, 64, 1, 1, 4), (32, 480, 64, 0, 1, 0), (32, 4, 64, 0, 0, 0), (64, 8, 128, 0, 0, 0),
])
def test_auto_range_matches_sequential_loop(oracle_mod, table, w, h, ll, layout, kind, frame):
    fr = oracle_mod.synth(1, w, h, ll, layout, kind, 0x7A1C, first_frame=frame)
    _, hsv = _hsv_image(oracle_mod, table, fr, w, h, ll, layout)
    rc, oa, _ = oracle_mod.run(fr, w, h, ll, layout, T0, auto_detect=True, preview=False)
    assert rc == 0 and oa["detect_written"] == 1
    got = [oa[k] for k in ("detect_hue", "detect_hue_tol", "detect_sat", "detect_sat_tol",
                           "detect_val", "detect_val_tol")]
    assert got == _auto_range_loop(hsv, w, h)


def _rgb565x(rgb):
    return ((rgb >> 19) & 0x1F) | ((rgb >> 5) & 0x7E0) | ((rgb << 8) & 0xF800)


def _preview_py(oracle_mod, table, fr, w, h, ll, layout, rng, ow, oh, oll):
    rgb, hsv = _hsv_image(oracle_mod, table, fr, w, h, ll, layout)
    f, t, e = oracle_mod.pack_range(rng)
    det = np.vectorize(lambda x: oracle_mod.lib().trik_oracle_detect(int(x), f, t, e))(hsv).astype(bool)
    shift = min(ow / w, oh / h)
    wi2wo = [int(i * shift) for i in range(w)]
    hi2ho = [int(i * shift) for i in range(h)]
    out = np.zeros((oh, oll), np.uint8)

    def put(r, c, v):
        out[r, 2 * c] = v & 0xFF
        out[r, 2 * c + 1] = (v >> 8) & 0xFF

    for r in range(h):  # proceedImageHsv: scan order, last writer wins
        for c in range(w):
            put(hi2ho[r], wi2wo[c], _rgb565x(0x00FFFF if det[r, c] else int(rgb[r, c])))

    def bound(c, r, v):
        c = min(max(c, 0), w - 1)
        r = min(max(r, 0), h - 1)
        put(hi2ho[r], wi2wo[c], _rgb565x(v))

    step, hh, hw = h // 6, h // 2, w // 2
    for col in (hw - 2 * step, hw - step, hw + step, hw + 2 * step):
        for adj in range(100):
            bound(col, hh - adj, 0xFF00FF)
            bound(col, hh + adj, 0xFF00FF)
    for row in (hh - 2 * step, hh - step, hh + step, hh + 2 * step):
        for adj in range(100):
            bound(hw - adj, row, 0xFF00FF)
            bound(hw + adj, row, 0xFF00FF)
    n = int(det.sum())
    if n:
        ys, xs = np.nonzero(det)
        cx, cy = int(xs.sum()) // n, int(ys.sum()) // n
        rad = math.ceil(float(np.sqrt(np.float32(n) / np.float32(3.1415927))))
        err, ey, ex, x, y = 1 - rad, 1, -2 * rad, rad, 0
        for dc, dr in ((0, rad), (0, -rad), (rad, 0), (-rad, 0)):
            bound(cx + dc, cy + dr, 0xFFFF00)
        while y < x:
            if err >= 0:
                x, ex = x - 1, ex + 2
                err += ex
            y, ey = y + 1, ey + 2
            err += ey
            for dc, dr in ((x, y), (x, -y), (-x, y), (-x, -y), (y, x), (y, -x), (-y, x), (-y, -x)):
                bound(cx + dc, cy + dr, 0xFFFF00)
    return out.reshape(-1)


@pytest.mark.parametrize("w,h,ll,layout,rng,ow,oh,oll", [
    (96, 48, 192, 0, T0, 48, 24, 96),
    (96, 48, 192, 0, T3, 60, 30, 121),
    (64, 48, 64, 1, T0, 64, 48, 128),
    (64, 48, 128, 0, (0, 359, 0, 100, 0, 100), 32, 40, 64),
])
def test_preview_matches_python_restatement(oracle_mod, table, w, h, ll, layout, rng, ow, oh, oll):
    fr = oracle_mod.synth(1, w, h, ll, layout, 1, 0x7A1C, first_frame=6)
    rc, _, pv = oracle_mod.run(fr, w, h, ll, layout, rng, out_width=ow, out_height=oh,
                               out_line_length=oll)
    assert rc == 0
    assert np.array_equal(pv, _preview_py(oracle_mod, table, fr, w, h, ll, layout, rng, ow, oh, oll))


def test_run_is_consistent_with_frame(oracle_mod):
    w, h, ll = 640, 480, 1280
    for kind, rng in ((0, T0), (1, T3)):
        fr = oracle_mod.synth(1, w, h, ll, 0, kind, 0x7A1C, first_frame=8)
        rc, oa, _ = oracle_mod.run(fr, w, h, ll, 0, rng)
        sums, _ = oracle_mod.frame(fr, w, h, ll, 0, [rng])
        assert rc == 0
        assert (oa["target_x"], oa["target_y"], oa["target_size"]) == oracle_mod.targets(sums[0], w, h)
        assert oa["detect_written"] == 0


def test_run_rejects_like_setup(oracle_mod):
    fr = np.zeros(64 * 64, np.uint8)
    assert oracle_mod.run(fr, 48, 4, 96, 0, T0)[0] == -1         # W % 32
    assert oracle_mod.run(fr, 32, 6, 64, 0, T0)[0] == -1         # H % 4
    assert oracle_mod.run(fr, 64, 64, 128, 0, T0)[0] == -1       # input smaller than H*lineLength
    assert oracle_mod.run(fr, 32, 4, 64, 0, T0, out_width=16, out_height=2, out_line_length=32)[0] == 0
