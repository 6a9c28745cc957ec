"""Generate tests/golden/oracle_golden.json from the CPU oracle.

Run from the repo root:  python tests/golden/make_golden.py

What the fixture holds (inputs are regenerated from seeds, not stored):
  * sha256 of the 2^24-entry per-(Y,U,V) table of (rgb << 32 | hsv), both
    derivations (they must be identical), plus 4096 sampled entries;
  * frame cases: (W, H, lineLength, layout, generator kind, seed, ranges) with
    the sha256 of the generated frame bytes (pins the generator) and the
    expected per-range {N, sumX, sumY} and {targetX, targetY, targetSize}.

These vectors are produced by the repo's own restatement of the reference
(the reference ships none and cannot be built here -- DESIGN.md section 3),
so they pin regressions and the GPU path, not the reference itself.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

# BASELINE ranges T0..T3 plus edge cases
RANGES = {
    "T0": (0, 30, 50, 100, 30, 100),
    "T1": (90, 150, 40, 100, 20, 100),
    "T2": (200, 260, 40, 100, 20, 100),
    "T3_wrap": (330, 20, 30, 100, 30, 100),
    "full": (0, 359, 0, 100, 0, 100),
    "empty_point": (10, 10, 100, 100, 100, 100),
    "from_eq_to": (120, 120, 0, 100, 0, 100),
    "wrap_adjacent": (2, 1, 0, 100, 0, 100),
    "wrap_359_0": (359, 0, 20, 100, 20, 100),
    "clamped_args": (400, 500, 200, 250, 0, 255),
    "grey": (0, 359, 0, 0, 0, 100),
    "dark": (0, 359, 0, 100, 0, 10),
}

CASES = [
    # name, W, H, lineLength, layout, kind, seed, frame, range names
    ("c1_ov7670_320x240_uniform", 320, 240, 320, O.LAYOUT_OV7670, 0, 0x7A1C, 0, ["T0"]),
    ("c1_ov7670_320x240_scene", 320, 240, 320, O.LAYOUT_OV7670, 1, 0x7A1C, 3, ["T0", "T1", "T2", "T3_wrap"]),
    ("c2_yuyv_640x480_uniform", 640, 480, 1280, O.LAYOUT_YUYV, 0, 0x7A1C, 0, ["T0"]),
    ("c2_yuyv_640x480_scene", 640, 480, 1280, O.LAYOUT_YUYV, 1, 0x7A1C, 1, list(RANGES)),
    ("c3_yuyv_640x480_frame4095", 640, 480, 1280, O.LAYOUT_YUYV, 0, 0x7A1C, 4095, ["T0", "T1", "T2", "T3_wrap"]),
    ("c4_yuyv_1280x720_scene", 1280, 720, 2560, O.LAYOUT_YUYV, 1, 0x7A1C, 7, ["T0", "T1"]),
    ("ragged_linelength_64x8", 64, 8, 160, O.LAYOUT_YUYV, 0, 99, 0, list(RANGES)),
    ("ragged_ov7670_96x12", 96, 12, 112, O.LAYOUT_OV7670, 0, 5, 2, list(RANGES)),
    ("minimal_32x4", 32, 4, 64, O.LAYOUT_YUYV, 0, 1, 0, list(RANGES)),
    ("empty_frame_640x0", 640, 0, 1280, O.LAYOUT_YUYV, 0, 1, 0, ["T0", "full"]),
]


# Whole BallDetector::run cases (trik_oracle_run): preview stream + OutArgs,
# with and without autoDetectHsv.  name, W, H, lineLength, layout, kind, seed,
# frame, range, auto, outW, outH, outLineLength
RUN_CASES = [
    ("run_640x480_scene_T0_auto", 640, 480, 1280, O.LAYOUT_YUYV, 1, 0x7A1C, 2, "T0", 1, 320, 240, 640),
    ("run_640x480_uniform_T3_auto", 640, 480, 1280, O.LAYOUT_YUYV, 0, 0x7A1C, 5, "T3_wrap", 1, 320, 240, 640),
    ("run_320x240_scene_full_scale0.625", 320, 240, 640, O.LAYOUT_YUYV, 1, 7, 0, "full", 0, 200, 150, 401),
    ("run_ov7670_320x240_scene_T1", 320, 240, 320, O.LAYOUT_OV7670, 1, 7, 4, "T1", 1, 160, 120, 320),
    ("run_32x480_zone_wrap", 32, 480, 64, O.LAYOUT_YUYV, 1, 3, 0, "T0", 1, 16, 240, 32),
    ("run_empty_point_no_circle", 320, 240, 640, O.LAYOUT_YUYV, 1, 3, 1, "empty_point", 1, 160, 120, 320),
]

# ov7670 line sensor (LSEQ:376-476): (name, w, h, ll, scene seed, x0, slope,
# val_from, val_to, band, out_w, out_h, out_ll); scene = oracle.line_scene
LINE_CASES = [
    ("line_320x240_dark_steady", 320, 240, 352, 1, None, 0.25, 0, 30, None, 160, 120, 320),
    ("line_640x480_portrait_out", 640, 480, 640, 2, 500, -0.5, 0, 30, None, 240, 320, 480),
    ("line_640x480_first_band_0_0", 640, 480, 640, 2, 500, -0.5, 0, 30, (0, 0), 320, 240, 640),
    ("line_320x240_bright_floor", 320, 240, 320, 3, 40, 0.0, 50, 100, None, 200, 150, 401),
    ("line_64x8_edge_line", 64, 8, 64, 4, 2, 0.0, 0, 30, None, 32, 4, 64),
    ("line_320x240_empty_range", 320, 240, 320, 5, None, 0.25, 80, 20, None, 160, 120, 320),
]

# ov7670 multi-blob sensor (OSEQ:516-602): scenes (oracle.blob_scene) and
# bitmap-driven frames (oracle.blob_frame of a random metapixel map)
BLOB_CASES = [
    ("blob_320x240_two_discs", "scene", 320, 240, 320, 1, 0.0, None, (0, 20, 80, 20, 50, 50), 160, 120, 320),
    ("blob_640x480_discs_salt", "scene", 640, 480, 704, 2, 0.01, None, (0, 20, 80, 20, 50, 50), 320, 240, 640),
    ("blob_160x120_meta_half", "meta", 160, 120, 176, 3, None, 0.5, (0, 20, 80, 20, 50, 50), 80, 60, 160),
    ("blob_160x120_meta_sparse", "meta", 160, 120, 160, 4, None, 0.12, (0, 20, 80, 20, 50, 50), 96, 72, 200),
    ("blob_320x240_meta_dense", "meta", 320, 240, 320, 5, None, 0.8, (0, 20, 80, 20, 50, 50), 160, 120, 320),
    ("blob_320x240_no_match", "scene", 320, 240, 320, 6, 0.0, None, (180, 10, 50, 10, 50, 10), 160, 120, 320),
]


def main():
    out = {"generator": "tests/golden/make_golden.py", "ranges": RANGES}
    a = O.yuv_table(closed=False)
    b = O.yuv_table(closed=True)
    assert np.array_equal(a, b), "derivations disagree"
    out["yuv_table_sha256"] = hashlib.sha256(a.tobytes()).hexdigest()
    rng = np.random.default_rng(20261015)
    idx = rng.integers(0, 1 << 24, 4096)
    out["yuv_table_samples"] = [[int(i), int(a[i])] for i in idx]
    lut43, lut255 = O.luts()
    out["lut43"] = lut43.tolist()
    out["lut255"] = lut255.tolist()
    out["packed_ranges"] = {k: list(O.pack_range(v)) for k, v in RANGES.items()}
    cases = []
    for name, w, h, ll, layout, kind, seed, fidx, rnames in CASES:
        fr = O.synth(1, w, h, ll, layout, kind, seed, first_frame=fidx)
        sums, _ = O.frame(fr, w, h, ll, layout, [RANGES[r] for r in rnames])
        tg = [list(O.targets(s, w, h)) for s in sums]
        cases.append({
            "name": name, "width": w, "height": h, "line_length": ll, "layout": layout,
            "kind": kind, "seed": seed, "frame": fidx, "ranges": rnames,
            "frame_sha256": hashlib.sha256(fr.tobytes()).hexdigest(),
            "sums": sums.tolist(), "targets": tg,
        })
    out["cases"] = cases
    runs = []
    for name, w, h, ll, layout, kind, seed, fidx, rname, auto, ow, oh, oll in RUN_CASES:
        fr = O.synth(1, w, h, ll, layout, kind, seed, first_frame=fidx)
        rc, oa, pv = O.run(fr, w, h, ll, layout, RANGES[rname], auto_detect=bool(auto),
                           out_width=ow, out_height=oh, out_line_length=oll)
        assert rc == 0, name
        runs.append({
            "name": name, "width": w, "height": h, "line_length": ll, "layout": layout,
            "kind": kind, "seed": seed, "frame": fidx, "range": rname, "auto": auto,
            "out_width": ow, "out_height": oh, "out_line_length": oll,
            "preview_sha256": hashlib.sha256(pv.tobytes()).hexdigest(), "outargs": oa,
        })
    out["runs"] = runs
    lines = []
    for name, w, h, ll, seed, x0, slope, vf, vt, band, ow, oh, oll in LINE_CASES:
        fr = O.line_scene(w, h, ll, seed, x0=x0, slope=slope)
        rc, oa, pv, sums, band_out = O.line_run(fr, w, h, ll, vf, vt, band=band, out_width=ow,
                                                out_height=oh, out_line_length=oll)
        assert rc == 0, name
        lines.append({
            "name": name, "width": w, "height": h, "line_length": ll, "seed": seed, "x0": x0,
            "slope": slope, "val_from": vf, "val_to": vt, "band": list(band) if band else None,
            "out_width": ow, "out_height": oh, "out_line_length": oll,
            "frame_sha256": hashlib.sha256(fr.tobytes()).hexdigest(),
            "preview_sha256": hashlib.sha256(pv.tobytes()).hexdigest(), "outargs": oa,
            "sums": sums.tolist(), "band_out": list(band_out),
        })
    out["line_runs"] = lines
    blobs = []
    for name, kind, w, h, ll, seed, noise, dens, hsv, ow, oh, oll in BLOB_CASES:
        if kind == "scene":
            fr = O.blob_scene(w, h, ll, seed, noise=noise)
        else:
            rng = np.random.default_rng(seed)
            meta = (rng.random((h // 4, w // 4)) < dens).astype(np.uint8)
            fr = O.blob_frame(meta, ll, seed=seed)
        r = O.blob_run(fr, w, h, ll, hsv=hsv, out_width=ow, out_height=oh, out_line_length=oll)
        assert r["rc"] == 0, name
        blobs.append({
            "name": name, "kind": kind, "width": w, "height": h, "line_length": ll, "seed": seed,
            "noise": noise, "density": dens, "hsv": list(hsv), "out_width": ow, "out_height": oh,
            "out_line_length": oll, "frame_sha256": hashlib.sha256(fr.tobytes()).hexdigest(),
            "targets": r["targets"].tolist(), "top": r["top"].tolist(), "n_labels": r["n_labels"],
            "preview_sha256": hashlib.sha256(r["preview"].tobytes()).hexdigest(),
            "labels_sha256": hashlib.sha256(r["labels"].tobytes()).hexdigest(),
        })
    out["blob_runs"] = blobs
    with open(os.path.join(HERE, "oracle_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(cases), "cases")


if __name__ == "__main__":
    main()
