"""The oracle's ov7670 multi-blob restatement (trik_oracle_blob_run; OSEQ =
trik/ov7670/object_sensor/include/internal/cv_ball_detector_seqpass.hpp, BMB =
cv_bitmap_builder_reference.hpp, CLU = cv_clusterizer_reference.hpp there) on
the CPU, against an independent Python restatement written from the reference
line by line: the per-pixel table for detection, the 4x4 bitmap (BMB:171-190),
Clusterizer::run with its vectors (CLU:44-202), std::sort by size with ties by
label, the 8 targets (OSEQ:563-590) and the preview (OSEQ:387-420, 548-580).
Parity unpinned (no reference fixture covers this path).
"""
import hashlib
import math

import numpy as np
import pytest

from test_oracle_run import _hsv_image, _rgb565x


def _wrap(v, adj, lo, hi):
    v += adj
    while v > hi:
        v -= hi - lo + 1
    while v < lo:
        v += hi - lo + 1
    return v


def _clip(v, adj, lo, hi):
    return min(max(v + adj, lo), hi)


def _range_py(hsv):
    """BMB:110-130 + resetHsvRange (BMB:62-77)."""
    h, ht, s, st, v, vt = hsv
    sc = lambda x, d: min(max((x * 255) // d, 0), 255)  # noqa: E731
    h0, h1 = sc(_wrap(h, -ht, 0, 359), 359), sc(_wrap(h, ht, 0, 359), 359)
    s0, s1 = sc(_clip(s, -st, 0, 100), 100), sc(_clip(s, st, 0, 100), 100)
    v0, v1 = sc(_clip(v, -vt, 0, 100), 100), sc(_clip(v, vt, 0, 100), 100)
    if h0 <= h1:
        return (v0 << 16) | (s0 << 8) | h0, (v1 << 16) | (s1 << 8) | h1, 0
    return (v0 << 16) | (s0 << 8) | ((h1 + 1) & 255), (v1 << 16) | (s1 << 8) | ((h0 - 1) & 255), 1


def _detect_py(hsv, rng):
    f, t, e = rng
    out = np.zeros(hsv.shape, np.int64)
    for k in range(3):  # cmpltu4 | cmpgtu4 per byte lane
        x = (hsv >> (8 * k)) & 255
        out |= (((x < ((f >> (8 * k)) & 255)) | (x > ((t >> (8 * k)) & 255))).astype(np.int64) << k)
    return out == e


def clusterize_py(meta):
    """Clusterizer::run (CLU:174-202) + postProcessing (CLU:115-127), literally."""
    bh, bw = meta.shape
    lab = [[0] * bw for _ in range(bh)]
    eq = [0]
    cl = [[0, 0, 0]]  # x, y, size
    for r in range(bh):
        for c in range(bw):
            if not meta[r, c]:
                continue
            a = [0, 0, 0, 0]
            if r != 0:
                a[2] = lab[r - 1][c]
                if c != 0:
                    a[1] = lab[r - 1][c - 1]
                if c != bw - 1:
                    a[3] = lab[r - 1][c + 1]
            if c != 0:
                a[0] = lab[r][c - 1]
            v = a[0]
            for n in range(1, 4):
                if (a[n] < v and a[n] != 0) or v == 0:
                    v = a[n]
            if v:
                lab[r][c] = v
                cl[v][0] += c
                cl[v][1] += r
                cl[v][2] += 1
                for ai in a:
                    if ai and not (ai == v or eq[ai] == eq[v]):
                        eq[ai] = eq[v]
            else:
                lab[r][c] = len(eq)
                eq.append(len(eq))
                cl.append([0, 0, 0])
    for i in range(len(eq)):
        if i != eq[i]:
            for k in range(3):
                cl[eq[i]][k] += cl[i][k]
            cl[i][2] = 0
    order = sorted(range(len(cl)), key=lambda i: (-cl[i][2], i))
    return np.array(lab, np.int64).reshape(bh, bw), [cl[i] for i in order], len(eq)


def blob_py(oracle_mod, table, fr, w, h, ll, hsv, ow, oh, oll):
    rgb, px_hsv = _hsv_image(oracle_mod, table, fr, w, h, ll, oracle_mod.LAYOUT_OV7670)
    det = _detect_py(px_hsv, _range_py(hsv))
    bw, bh = w // 4, h // 4
    meta = det.reshape(bh, 4, bw, 4).sum(axis=(1, 3)) > 2
    lab, clusters, n = clusterize_py(meta)
    out = np.zeros((oh, oll), np.uint8)
    shift = min(ow / w, oh / h)
    wi2wo = [int(i * shift) for i in range(w)]
    hi2ho = [int(i * shift) for i in range(h)]

    def put(r, c, v):
        out[r, 2 * c] = v & 0xFF
        out[r, 2 * c + 1] = (v >> 8) & 0xFF

    for r in range(h):
        for c in range(w):
            put(hi2ho[r], wi2wo[c], _rgb565x(0x00FFFF if lab[r // 4, c // 4] else int(rgb[r, c])))

    def bound(c, r, v):
        put(hi2ho[min(max(r, 0), h - 1)], wi2wo[min(max(c, 0), w - 1)], _rgb565x(v))

    step, hh, hw = h // 6, h // 2, w // 2
    for col in (hw - step, hw + step, hw - 2 * step, hw + 2 * step):
        for adj in range(100):
            bound(col, hh - adj, 0xFF00FF)
            bound(col, hh + adj, 0xFF00FF)
    for row in (hh - step, hh + step, hh - 2 * step, hh + 2 * step):
        for adj in range(100):
            bound(hw - adj, row, 0xFF00FF)
            bound(hw + adj, row, 0xFF00FF)
    targets = np.zeros((8, 3), np.int64)
    top = np.zeros((8, 3), np.int64)
    for i in range(8):
        x_, y_, s_ = clusters[i] if i < len(clusters) else (0, 0, 0)
        if i < len(clusters):
            top[i] = (s_, x_, y_)
        root = int(math.sqrt(float(np.float32(s_ & 0xFFFF))))
        radius = math.ceil(float(np.float32(root) / np.float32(3.1415927)))
        size = (radius * 400) // (bw + bh)
        if size > 4:
            x, y = (x_ // (s_ + 1)) * 4, (y_ // (s_ + 1)) * 4
            for dc in (-1, 0, 1):
                for dr in (-1, 0, 1):
                    bound(x + dc, y + dr, 0xFF0000)
            tx = int(((x - w // 2) * 200) / w)  # C division truncates toward zero
            ty = int(((y - h // 2) * 200) / h)
            i8 = lambda v: (v + 128) % 256 - 128  # noqa: E731  (XDAS_Int8 store wraps)
            targets[i] = (i8(tx), i8(ty), size & 255)
    return {"meta": meta.astype(np.uint8), "labels": lab, "top": top, "targets": targets,
            "n_labels": n, "preview": out.reshape(-1)}


@pytest.mark.parametrize("case", [
    ("scene", 160, 120, 176, 1, 0.0),
    ("scene", 96, 64, 96, 2, 0.02),
    ("meta", 0.1, 40, 30, 3),
    ("meta", 0.5, 40, 30, 4),
    ("meta", 0.85, 24, 20, 5),
    ("meta", 0.5, 8, 1, 6),
    ("meta", 0.5, 8, 9, 7),
])
def test_blob_run_matches_python_restatement(oracle_mod, table, case):
    if case[0] == "scene":
        _, w, h, ll, seed, noise = case
        fr = oracle_mod.blob_scene(w, h, ll, seed, noise=noise)
    else:
        _, dens, bw, bh, seed = case
        rng = np.random.default_rng(seed)
        meta = (rng.random((bh, bw)) < dens).astype(np.uint8)
        w, h, ll = 4 * bw, 4 * bh, 4 * bw + 16
        fr = oracle_mod.blob_frame(meta, ll, seed=seed)
    ow, oh, oll = w // 2 + 8, h // 2, w + 20
    r = oracle_mod.blob_run(fr, w, h, ll, hsv=oracle_mod.RED_HSV, out_width=ow, out_height=oh,
                            out_line_length=oll)
    assert r["rc"] == 0
    ref = blob_py(oracle_mod, table, fr, w, h, ll, oracle_mod.RED_HSV, ow, oh, oll)
    assert np.array_equal(r["meta"], ref["meta"])
    assert np.array_equal(r["labels"], ref["labels"])
    assert r["n_labels"] == ref["n_labels"]
    assert np.array_equal(r["top"], ref["top"])
    assert np.array_equal(r["targets"], ref["targets"])
    assert np.array_equal(r["preview"], ref["preview"])


def test_blob_range_packing(oracle_mod):
    for hsv in [(0, 20, 80, 20, 50, 50), (180, 30, 50, 50, 50, 50), (350, 30, 10, 20, 0, 0),
                (10, 0, 100, 0, 100, 0), (359, 359, 0, 100, 0, 100), (200, 400, 50, 200, 50, 70)]:
        assert oracle_mod.blob_range(hsv) == _range_py(hsv), hsv


def test_blob_state_is_sticky(oracle_mod):
    fr = oracle_mod.blob_scene(160, 120, 160, 9)
    a = oracle_mod.blob_run(fr, 160, 120, 160, hsv=oracle_mod.RED_HSV)
    b = oracle_mod.blob_run(fr, 160, 120, 160, hsv=None, state=a["state"])
    z = oracle_mod.blob_run(fr, 160, 120, 160, hsv=None)  # never set: all-zero range
    assert np.array_equal(a["targets"], b["targets"]) and np.array_equal(a["preview"], b["preview"])
    assert a["meta"].sum() > 0 and z["meta"].sum() == 0


def test_golden_blob_runs(oracle_mod, golden):
    assert len(golden["blob_runs"]) >= 5
    for c in golden["blob_runs"]:
        if c["kind"] == "scene":
            fr = oracle_mod.blob_scene(c["width"], c["height"], c["line_length"], c["seed"],
                                       noise=c["noise"])
        else:
            rng = np.random.default_rng(c["seed"])
            meta = (rng.random((c["height"] // 4, c["width"] // 4)) < c["density"]).astype(np.uint8)
            fr = oracle_mod.blob_frame(meta, c["line_length"], seed=c["seed"])
        assert hashlib.sha256(fr.tobytes()).hexdigest() == c["frame_sha256"], c["name"]
        r = oracle_mod.blob_run(fr, c["width"], c["height"], c["line_length"], hsv=tuple(c["hsv"]),
                                out_width=c["out_width"], out_height=c["out_height"],
                                out_line_length=c["out_line_length"])
        assert r["rc"] == 0
        assert r["targets"].tolist() == c["targets"], c["name"]
        assert r["top"].tolist() == c["top"], c["name"]
        assert r["n_labels"] == c["n_labels"], c["name"]
        assert hashlib.sha256(r["preview"].tobytes()).hexdigest() == c["preview_sha256"], c["name"]
        assert hashlib.sha256(r["labels"].tobytes()).hexdigest() == c["labels_sha256"], c["name"]


def test_blob_run_rejects(oracle_mod):
    fr = np.zeros(2 * 64 * 64, np.uint8)
    assert oracle_mod.blob_run(fr, 48, 4, 48, hsv=oracle_mod.RED_HSV)["rc"] == -1   # W % 32
    assert oracle_mod.blob_run(fr, 32, 6, 32, hsv=oracle_mod.RED_HSV)["rc"] == -1   # H % 4
    assert oracle_mod.blob_run(fr[:64 * 64], 64, 64, 64, hsv=oracle_mod.RED_HSV)["rc"] == -1  # planes
