"""CPU tests of the oracle (test infrastructure) against the fixed points it is
pinned by: TI intrinsic semantics, the two independent derivations, the SURVEY
Appendix A known-answer table and the committed golden fixtures."""
import hashlib

import numpy as np
import pytest


# --- per-intrinsic unit tests (hand-derived from TI's documented C64x+ semantics) ---
@pytest.mark.parametrize("name,args,expect", [
    ("mpyu4ll", (0x01020304, 0x05060708), 0x0005000C00150020),
    ("dotpus4", (0xFF010203, 0x80FF0102), -32633),
    ("add2", (0xFFFF0001, 0x00010001), 0x00000002),
    ("shr2", (0x8000FFC0, 6), 0xFE00FFFF),
    ("spacku4", (0x01FFFF80, 0x00FF7FFF), 0xFF00FFFF),
    ("cmpeq2", (0x00050007, 0x00050008), 2),
    ("dotpn2", (0x00030004, 0xFFFE0005), -26),
    ("packh4", (0xAABBCCDD, 0x11223344), 0xAACC1133),
    ("cmpltu4", (0x01FF0080, 0x02FE0180), 0b1010),
    ("cmpgtu4", (0x01FF0080, 0x02FE0180), 0b0100),
    ("swap4", (0x11223344,), 0x22114433),
    ("unpkhu4", (0xAABBCCDD,), 0x00AA00BB),
    ("unpklu4", (0xAABBCCDD,), 0x00CC00DD),
    ("packh2", (0x12345678, 0x9ABCDEF0), 0x12349ABC),
    ("packlh2", (0x12345678, 0x9ABCDEF0), 0x56789ABC),
    ("pack2", (0x12345678, 0x9ABCDEF0), 0x5678DEF0),
    ("packhl2", (0x12345678, 0x9ABCDEF0), 0x1234DEF0),
    ("clr", (0xFFFFFFFF, 16, 31), 0x0000FFFF),
    ("clr", (0xFFFFFFFF, 8, 31), 0x000000FF),
    ("maxu4", (0x01FF7F80, 0x02FE8070), 0x02FF8080),
    ("minu4", (0x01FF7F80, 0x02FE8070), 0x01FE7F70),
])
def test_intrinsic(oracle_mod, name, args, expect):
    assert getattr(oracle_mod.lib(), "trik_c64x_" + name)(*args) == expect


def test_luts(oracle_mod, golden):
    lut43, lut255 = oracle_mod.luts()
    assert lut43[0] == 0 and lut255[0] == 0
    assert all(lut43[i] == 11008 // i and lut255[i] == 65280 // i for i in range(1, 256))
    assert lut43.tolist() == golden["lut43"] and lut255.tolist() == golden["lut255"]


def test_derivations_agree_all_yuv_pixel0(oracle_mod, table):
    """Intrinsic-level restatement == closed form, all 2^24 (Y,U,V), pixel 0."""
    closed = oracle_mod.yuv_table(closed=True)
    assert np.array_equal(table, closed)


def test_derivations_agree_all_yuv_pixel1(oracle_mod):
    """Pixel 1 of the pair (Y in byte 2) with an unrelated pixel-0 luma."""
    L = oracle_mod.lib()
    rng = np.random.default_rng(7)
    for _ in range(20000):
        y0, u, y1, v = (int(x) for x in rng.integers(0, 256, 4))
        p0, p1 = oracle_mod.pair_rgb(y0 | u << 8 | y1 << 16 | v << 24)
        assert p0 == L.trik_oracle_rgb_closed(y0, u, v)
        assert p1 == L.trik_oracle_rgb_closed(y1, u, v)


def test_hsv_derivations_agree_all_rgb(oracle_mod):
    L = oracle_mod.lib()
    rng = np.random.default_rng(11)
    for rgb in list(rng.integers(0, 1 << 24, 200000)) + [0, 0xFFFFFF, 0x00FF00, 0xFF0000, 0x0000FF]:
        rgb = int(rgb)
        assert L.trik_oracle_hsv_c64x(rgb) == L.trik_oracle_hsv_closed(rgb), hex(rgb)


KATS = [  # (Y,U,V) -> (R,G,B) / (H,S,V)
    ((16, 128, 128), (0, 0, 0), (85, 0, 0)),
    ((235, 128, 128), (253, 253, 253), (85, 0, 253)),
    ((81, 90, 240), (253, 0, 0), (0, 254, 253)),
    ((145, 54, 34), (0, 254, 0), (85, 254, 254)),
    ((41, 240, 110), (0, 0, 255), (170, 255, 255)),
    ((237, 255, 128), (255, 206, 255), (213, 49, 255)),
    ((238, 255, 128), (255, 207, 0), (34, 255, 255)),
    ((255, 255, 128), (255, 227, 0), (38, 255, 255)),
    ((0, 0, 0), (0, 135, 0), (85, 254, 135)),
    ((255, 255, 255), (255, 123, 0), (20, 255, 255)),
]


@pytest.mark.parametrize("yuv,rgb,hsv", KATS)
def test_appendix_a_kats(table, yuv, rgb, hsv):
    y, u, v = yuv
    e = int(table[y | u << 8 | v << 16])
    r, h = e >> 32, e & 0xFFFFFFFF
    assert ((r >> 16) & 255, (r >> 8) & 255, r & 255) == rgb
    assert (h & 255, (h >> 8) & 255, (h >> 16) & 255) == hsv


def test_b_wrap_count(table):
    """SURVEY 7 hard part 1: B wraps to 0 for exactly 27,136 (Y,U,V) triples."""
    idx = np.arange(1 << 24, dtype=np.int64)
    y, u = idx & 255, (idx >> 8) & 255
    wraps = (129 * u + 74 * y - 17672) >= 32768
    assert int(wraps.sum()) == 27136
    assert np.all(((table[wraps] >> 32) & 255) == 0)


def test_table_digest(table, golden):
    assert hashlib.sha256(table.tobytes()).hexdigest() == golden["yuv_table_sha256"]
    for i, v in golden["yuv_table_samples"]:
        assert int(table[i]) == v


def test_pack_range(oracle_mod, golden):
    for name, r in golden["ranges"].items():
        assert list(oracle_mod.pack_range(tuple(r))) == golden["packed_ranges"][name], name


def test_golden_frames(oracle_mod, golden):
    for c in golden["cases"]:
        fr = oracle_mod.synth(1, c["width"], c["height"], c["line_length"], c["layout"],
                              c["kind"], c["seed"], first_frame=c["frame"])
        assert hashlib.sha256(fr.tobytes()).hexdigest() == c["frame_sha256"], c["name"]
        rs = [tuple(golden["ranges"][r]) for r in c["ranges"]]
        sums, _ = oracle_mod.frame(fr, c["width"], c["height"], c["line_length"], c["layout"], rs)
        assert sums.tolist() == c["sums"], c["name"]
        for s, t in zip(sums, c["targets"]):
            assert list(oracle_mod.targets(s, c["width"], c["height"])) == t


def test_frame_matches_per_pixel_table(oracle_mod, table):
    """Frame-level sums == sums rebuilt from the per-pixel table (independent path)."""
    w, h, ll = 64, 16, 128
    fr = oracle_mod.synth(1, w, h, ll, oracle_mod.LAYOUT_YUYV, 0, 3)
    r = (0, 30, 50, 100, 30, 100)
    sums, mask = oracle_mod.frame(fr, w, h, ll, oracle_mod.LAYOUT_YUYV, [r], want_mask=True)
    f, t, e = oracle_mod.pack_range(r)
    L = oracle_mod.lib()
    px = fr.reshape(h, ll)[:, : 2 * w].reshape(h, w // 2, 4).astype(np.int64)
    n = sx = sy = 0
    for yy in range(h):
        for q in range(w // 2):
            y0, u, y1, v = px[yy, q]
            for k, ly in enumerate((y0, y1)):
                hsv = int(table[ly | u << 8 | v << 16]) & 0xFFFFFFFF
                d = L.trik_oracle_detect(hsv, f, t, e)
                assert d == (mask[yy, 2 * q + k] & 1)
                n += d; sx += d * (2 * q + k); sy += d * yy
    assert sums.tolist() == [[n, sx, sy]]


def test_rejects_bad_geometry(oracle_mod):
    fr = np.zeros(64 * 8, np.uint8)
    with pytest.raises(ValueError):
        oracle_mod.frame(fr, 48, 4, 96, 0, [(0, 30, 0, 100, 0, 100)])   # W % 32
    with pytest.raises(ValueError):
        oracle_mod.frame(fr, 32, 6, 64, 0, [(0, 30, 0, 100, 0, 100)])   # H % 4
    with pytest.raises(ValueError):
        oracle_mod.frame(fr, 32, 16, 64, 0, [(0, 30, 0, 100, 0, 100)])  # buffer too small


def test_epilogue_edges(oracle_mod):
    # N = 0 -> zeros; full 640x480 frame detected -> centre, size from the radius
    assert oracle_mod.targets([0, 0, 0], 640, 480) == (0, 0, 0)
    n = 640 * 480
    sx = 480 * (639 * 640 // 2)
    sy = 640 * (479 * 480 // 2)
    x, y, s = oracle_mod.targets([n, sx, sy], 640, 480)
    assert (x, y) == (0, 0)  # cx=319 -> (319-320)*200/640 truncates to 0
    assert s == (313 * 400) // 1120


# --- the clean-room scalar CPU baseline (bench.py cpu_baseline) equals the oracle ---
@pytest.mark.parametrize("layout,kind,n_ranges", [(0, 0, 4), (0, 1, 4), (1, 1, 2), (0, 1, 12), (1, 0, 1)])
def test_cpu_baseline_equals_oracle(oracle_mod, layout, kind, n_ranges):
    o = oracle_mod
    ranges = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100), (200, 260, 40, 100, 20, 100),
              (330, 20, 30, 100, 30, 100), (0, 359, 0, 100, 0, 100), (10, 10, 0, 100, 0, 100),
              (359, 0, 0, 100, 0, 100), (45, 300, 5, 95, 5, 95), (120, 121, 50, 51, 50, 51),
              (0, 359, 0, 0, 0, 0), (180, 179, 0, 100, 0, 100), (-5, 400, -1, 200, -1, 200)][:n_ranges]
    w, h = 320, 240
    ll = 2 * w if layout == o.LAYOUT_YUYV else w + 32
    stride = h * ll * (2 if layout == o.LAYOUT_OV7670 else 1)
    frames = o.synth(6, w, h, ll, layout, kind, 0x51 + kind)
    want, _ = o.batch(frames, stride, 6, w, h, ll, layout, ranges)
    got = o.cpu_batch(frames, stride, 6, w, h, ll, layout, ranges, n_threads=3)
    assert np.array_equal(got, want)


# --- the webcam line sensor restatement (trik_oracle_wline_run, LSEQW) ---
@pytest.mark.parametrize("vf,vt", [(0, 30), (50, 100), (80, 20), (0, 100)])
def test_wline_sums_are_the_object_sensor_sums_of_its_range(oracle_mod, vf, vt):
    """LSEQW's detection is the object sensor's with H 0..359, S 0..100 (both
    0..255 after scaling, LSEQW:345-364): its {N, sumX, sumY} equal
    trik_oracle_frame's for that range; the OutArgs follow LSEQW:405-417."""
    o = oracle_mod
    w, h, ll = 320, 240, 672
    fr = o.wline_scene(w, h, ll, 5, slope=-0.3)
    rc, oa, pv, sums = o.wline_run(fr, w, h, ll, vf, vt, out_width=160, out_height=120)
    assert rc == 0
    want, _ = o.frame(fr, w, h, ll, o.LAYOUT_YUYV, [(0, 359, 0, 100, vf, vt)])
    assert sums.tolist() == want[0].tolist()
    n, sx = int(sums[0]), int(sums[1])
    if n > 10:
        tx = (sx & 0xFFFFFFFF) // n
        assert oa["target_x"] == int(np.int8(int(((tx - w // 2) * 200) / w)))
        assert oa["target_size"] == (n * 100) // (w * h) % 256
    else:
        assert (oa["target_x"], oa["target_size"]) == (0, 0)
    assert oa["target_y"] == 0
    # thin lines (magenta, 0xff00ff -> RGB565X 0x1ff8 little-endian) over every output row
    img = pv.reshape(120, 320)
    for c in (w // 2 - 80, w // 2 - 40, w // 2 + 40, w // 2 + 80):
        oc = int(c * 0.5)
        if n <= 10 or abs(c - (sx & 0xFFFFFFFF) // n) > 3:
            assert (img[:, 2 * oc] == 0x1f).all() and (img[:, 2 * oc + 1] == 0xf8).all(), c


def test_wline_rejects_and_empty(oracle_mod):
    o = oracle_mod
    assert o.wline_run(np.zeros(64 * 8, np.uint8), 48, 4, 96, 0, 30)[0] != 0      # W % 32
    assert o.wline_run(np.zeros(64 * 8, np.uint8), 32, 6, 64, 0, 30)[0] != 0      # H % 4
    assert o.wline_run(np.zeros(64 * 8, np.uint8), 32, 16, 64, 0, 30)[0] != 0     # short input
    rc, oa, pv, sums = o.wline_run(np.zeros(16, np.uint8), 0, 0, 0, 0, 30, out_width=0, out_height=0)
    assert rc == 0 and sums.tolist() == [0, 0, 0] and not pv.any()
