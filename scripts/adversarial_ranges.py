"""Chroma-run vs stripe kernel time for range sets of increasing exact-path
share (uniform C3 frames), and for the bench ranges on frames concentrated on
the chromas the chroma-run tables describe worst (window / exception
chromas), to place and check the AUTO selector (development only).

usage (GPU box): python scripts/adversarial_ranges.py [frames]
One line per case: the builder's expected flagged-word share (uniform
input), the measured share of the frames where it differs, then each
hot-kernel setting's kernel and ms per batch (trik_hsv_batch_sums, HIP events;
median of 3 passes in rotated order, 40 synchronised warm-up calls per
setting and pass).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "trik-media-sensors-dsp_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]
import trik_hsv  # noqa: E402

BENCH = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
         (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]
# expected exact-path shares from the numpy model of the builder
# (tests/test_chroma_model.py), uniform input
SETS = {
    "bench 4 ranges (0.029)": BENCH,
    "bench3 + hue0-90 S30-40 (0.07)": BENCH[:3] + [(0, 90, 30, 40, 0, 100)],
    "bench3 + hue0-135 S30-40 (~0.10)": BENCH[:3] + [(0, 135, 30, 40, 0, 100)],
    "bench3 + V20-40 (0.14)": BENCH[:3] + [(0, 359, 0, 100, 20, 40)],
    "bench2 + S30-40 (0.16)": BENCH[:2] + [(0, 359, 30, 40, 0, 100)],
    "bench3 + hue0-270 S30-40 (~0.20)": BENCH[:3] + [(0, 270, 30, 40, 0, 100)],
    "bench3 + S30-35 (0.23)": BENCH[:3] + [(0, 359, 30, 35, 0, 100)],
    "bench3 + S50-100 (0.25)": BENCH[:3] + [(0, 359, 50, 100, 0, 100)],
    "bench3 + S30-40 (0.27)": BENCH[:3] + [(0, 359, 30, 40, 0, 100)],
    "bench3 + S20-40 (0.32)": BENCH[:3] + [(0, 359, 20, 40, 0, 100)],
    "hue0-30 S50-60 (T=1)": [(0, 30, 50, 60, 0, 100)],
    "2 x hue60 S30-60": [(0, 60, 30, 60, 20, 100), (120, 180, 30, 60, 20, 100)],
    "two S bands": [(0, 359, 20, 30, 0, 100), (0, 359, 60, 70, 0, 100)],
    "four S bands": [(0, 359, 20, 25, 0, 100), (0, 359, 40, 45, 0, 100),
                     (0, 359, 60, 65, 0, 100), (0, 359, 80, 85, 0, 100)],
}


def concentrated_frames(F, W, H, kinds, seed=5):
    """Frames whose chromas are drawn from the bench set's window and/or
    exception chromas (the numpy model of the builder), Y uniform; and the
    flagged-word share those frames give."""
    import oracle as om
    import test_chroma_model as tm

    P = tm.profiles(om, BENCH)
    runs, _, _ = tm.build(P)
    b1, b2 = runs & 255, runs >> 8
    exc = runs == tm.KEXC
    win = ~exc & (b1 > b2 + 1)
    pick = np.zeros(65536, bool)
    if "window" in kinds:
        pick |= win
    if "exception" in kinds:
        pick |= exc
    chromas = np.nonzero(pick)[0].astype(np.uint32)
    L = np.where(exc, 256, np.maximum(b1 - b2 - 1, 0))
    share = float(np.mean(1 - (1 - L[chromas] / 256.0) ** 2))
    rng = np.random.default_rng(seed)
    n = F * H * W // 2
    c = chromas[rng.integers(0, len(chromas), n)]
    y = rng.integers(0, 256, (n, 2), dtype=np.uint32)
    words = y[:, 0] | ((c & 255) << 8) | (y[:, 1] << 16) | ((c >> 8) << 24)
    return words.astype("<u4").view(np.uint8), share


def time_case(frames, F, W, H, ranges, reps=20, warm=40, passes=3, seed=0):
    """Each hot-kernel setting on its own handle (AUTO's measured-share state
    is per handle), all built before any timing; then `passes` passes, each
    in a rotated order (pass p starts at setting p), every setting given the
    same `warm` synchronised warm-up calls before its `reps` timed calls (HIP
    events); the median over the passes.  (Round 4's table timed the settings
    in a fixed order -- forced chroma right after the cold table build with 5
    warm-ups, AUTO last with 40 -- so clock transients decided the ratios.)"""
    ll = 2 * W
    stream = torch.cuda.current_stream()
    kinds = (trik_hsv.HOT_CHROMA, trik_hsv.HOT_STRIPE, trik_hsv.HOT_AUTO)
    dets = {}
    sums = torch.zeros((F, len(ranges), 3), dtype=torch.int64, device=frames.device)
    expected = None
    for hot in kinds:
        det = trik_hsv.Detector(hot=hot)
        det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
        torch.cuda.synchronize()
        if hot == trik_hsv.HOT_CHROMA:
            expected = det.chroma_flagged_share()
        dets[hot] = det
    times = {hot: [] for hot in kinds}
    ran = {}
    for p in range(passes):
        order = kinds[p % 3:] + kinds[:p % 3]
        for hot in order:
            det = dets[hot]
            # warm-up, synchronised per call: AUTO reads the measured share
            # back every few launches (trik_hsv_abi.cpp: probe_measured)
            for _ in range(warm):
                det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
                torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times[hot].append(e0.elapsed_time(e1) / reps)
            r = {trik_hsv.HOT_CHROMA: "chroma", trik_hsv.HOT_STRIPE: "stripe",
                 trik_hsv.HOT_MIXED: "mixed"}.get(det.last_hot_kernel(), "?")
            if hot == trik_hsv.HOT_AUTO:
                r += f"[m={det.chroma_measured_share():.3f}]"
            ran[hot] = r
    out = []
    for hot in kinds:
        t = sorted(times[hot])
        out.append((["auto", "stripe", "chroma"][hot], ran[hot], t[len(t) // 2]))
    for det in dets.values():
        det.close()
    return expected, out


def line(name, F, W, H, expected, res, measured=None):
    ll = 2 * W
    parts = [f"{name:36s}", f"share {expected:.3f}"]
    if measured is not None:
        parts.append(f"(frames {measured:.3f})")
    t = {k: ms for k, _, ms in res}
    for k, ran, ms in res:
        parts.append(f"{k}->{ran} {ms:.3f} ms ({100 * F * H * ll / (ms * 1e-3) / 8e12:.1f} %)")
    best = min(t["chroma"], t["stripe"])
    parts.append(f"auto/best {t['auto'] / best:.2f}")
    print("  ".join(parts), flush=True)


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    W, H = 640, 480
    ll = 2 * W
    dev = torch.device("cuda", 0)
    frames = torch.empty(F * H * ll, dtype=torch.uint8, device=dev)
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, 0, 0x7A1C)
    for name, ranges in SETS.items():
        expected, res = time_case(frames, F, W, H, ranges)
        line(name, F, W, H, expected, res)
    for kinds in (("window",), ("exception",), ("window", "exception")):
        host, share = concentrated_frames(F, W, H, kinds)
        frames.copy_(torch.from_numpy(host))
        del host
        expected, res = time_case(frames, F, W, H, BENCH)
        line("bench, frames on " + "+".join(kinds) + " chromas", F, W, H, expected, res, share)


if __name__ == "__main__":
    main()
