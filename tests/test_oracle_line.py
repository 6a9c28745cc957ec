"""The oracle's ov7670 line-sensor restatement (trik_oracle_line_run, LSEQ =
trik/ov7670/line_sensor/include/internal/cv_line_detector_seqpass.hpp) on the
CPU: against the committed golden runs, and against an independent numpy
restatement built on the per-pixel table (detection by V only in columns
5..W-5, LSEQ:283-299, 391-414; the overlays of LSEQ:88-130, 433-467; the
OutArgs of LSEQ:452-474).  Parity unpinned (no reference fixture covers the
line sensor); the per-pixel arithmetic it uses is the pinned one.
"""
import hashlib

import numpy as np
import pytest

from test_oracle_run import _hsv_image, _rgb565x


def test_golden_line_runs(oracle_mod, golden):
    assert len(golden["line_runs"]) >= 6
    for c in golden["line_runs"]:
        fr = oracle_mod.line_scene(c["width"], c["height"], c["line_length"], c["seed"], x0=c["x0"],
                                   slope=c["slope"])
        assert hashlib.sha256(fr.tobytes()).hexdigest() == c["frame_sha256"], c["name"]
        rc, oa, pv, sums, band = oracle_mod.line_run(
            fr, c["width"], c["height"], c["line_length"], c["val_from"], c["val_to"], band=c["band"],
            out_width=c["out_width"], out_height=c["out_height"], out_line_length=c["out_line_length"])
        assert rc == 0
        assert hashlib.sha256(pv.tobytes()).hexdigest() == c["preview_sha256"], c["name"]
        assert oa == c["outargs"], c["name"]
        assert sums.tolist() == c["sums"], c["name"]
        assert list(band) == c["band_out"], c["name"]


def _scale_val(v):
    return min(max((v * 255) // 100, 0), 255)


def line_py(oracle_mod, table, fr, w, h, ll, vf, vt, band, ow, oh, oll):
    """LineDetector::run restated with numpy + plain loops for the overlays."""
    rgb, hsv = _hsv_image(oracle_mod, table, fr, w, h, ll, oracle_mod.LAYOUT_OV7670)
    val = hsv >> 16
    cols = np.arange(w)
    win = (cols >= 5) & (cols <= w - 5)
    det = (val >= _scale_val(vf)) & (val <= _scale_val(vt)) & win[None, :]
    per_row = det.sum(1)
    n = int(per_row.sum())
    sx = int((det * cols[None, :]).sum())
    rows = np.arange(h)
    cross = int(per_row[(rows >= band[0]) & (rows <= band[1])].sum())

    shift = min(ow / w, oh / h)
    wi2wo = [int(i * shift) for i in range(w)]
    hi2ho = [int(i * shift) for i in range(h)]
    out = np.zeros((oh, oll), np.uint8)

    def put(r, c, v):
        out[r, 2 * c] = v & 0xFF
        out[r, 2 * c + 1] = (v >> 8) & 0xFF

    for r in range(h):
        for c in range(5, w - 4):  # only window pixels are written (LSEQ:288-291)
            put(hi2ho[r], wi2wo[c], _rgb565x(0x00FFFF if det[r, c] else int(rgb[r, c])))

    def bound(c, r, v):
        put(hi2ho[min(max(r, 0), h - 1)], wi2wo[min(max(c, 0), w - 1)], _rgb565x(v))

    step, hw, hh = 40, w // 2, h // 2
    for col in (hw - step, hw + step, hw - 2 * step, hw + 2 * step):
        for adj in range(h):
            bound(col, adj, 0xFF00FF)
    for row in (hh, hh + 2 * step):
        for adj in range(w):
            bound(adj, row, 0xFF0000)
    t = {"target_x": 0, "target_y": 0, "target_size": 0}
    if n > 10:
        cx = sx // n
        for adj in range(h):
            for d in (-1, 0, 1):
                bound(cx + d, adj, 0xFF0000)
        t = {"target_x": int(np.int8(((cx - w // 2) * 200) // w if cx >= w // 2
                                     else -(((w // 2 - cx) * 200) // w))),
             "target_y": int(np.int8(np.uint32(cross * 100) // np.uint32(w * 80))),
             "target_size": int(np.uint8((n * 100) // (w * h)))}
    return t, out.reshape(-1), [n, sx, cross]


@pytest.mark.parametrize("w,h,ll,seed,x0,slope,vf,vt,band,ow,oh,oll", [
    (96, 48, 96, 11, None, 0.25, 0, 30, None, 48, 24, 96),
    (96, 48, 128, 12, 10, 0.5, 0, 30, (0, 47), 60, 30, 121),
    (64, 40, 64, 13, 50, -0.25, 40, 100, None, 64, 40, 128),
    (128, 120, 128, 14, 60, 0.0, 0, 30, (70, 60), 64, 60, 128),
    (64, 8, 64, 15, 0, 0.0, 0, 100, None, 32, 4, 64),
])
def test_line_run_matches_python_restatement(oracle_mod, table, w, h, ll, seed, x0, slope, vf, vt,
                                             band, ow, oh, oll):
    fr = oracle_mod.line_scene(w, h, ll, seed, x0=x0, slope=slope, line_w=9)
    b = band if band is not None else (h // 2, h // 2 + 80)
    rc, oa, pv, sums, band_out = oracle_mod.line_run(fr, w, h, ll, vf, vt, band=b, out_width=ow,
                                                     out_height=oh, out_line_length=oll)
    assert rc == 0
    t, pv_py, sums_py = line_py(oracle_mod, table, fr, w, h, ll, vf, vt, b, ow, oh, oll)
    assert sums.tolist() == sums_py
    assert {k: oa[k] for k in t} == t
    assert oa["detect_written"] == 0
    assert band_out == (h // 2, h // 2 + 80)
    assert np.array_equal(pv, pv_py)


def test_line_run_rejects(oracle_mod):
    fr = np.zeros(2 * 64 * 64, np.uint8)
    assert oracle_mod.line_run(fr, 48, 4, 48, 0, 30)[0] == -1     # W % 32 (LSEQ:328-332)
    assert oracle_mod.line_run(fr, 32, 6, 32, 0, 30)[0] == -1     # H % 4
    assert oracle_mod.line_run(fr[: 64 * 64 + 8], 64, 64, 64, 0, 30)[0] == -1  # needs both planes
    assert oracle_mod.line_run(fr, 32, 4, 32, 0, 30, out_width=16, out_height=2, out_line_length=32)[0] == 0
