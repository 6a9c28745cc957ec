"""Does a small kernel on a second stream run while the hot kernel runs?
(bench.py's N > 1 step puts step k's all-reduce on a second
stream "while step k+1's kernel runs".)  Development measurement on one GPU.

The C3 step (trik_hsv_process_batch_totals: one chroma_kernel launch, one
workgroup of 1024 lanes and ~160 KiB of LDS per CU, 4 waves on every SIMD)
runs back to back on stream A; after each step, stream B waits for it (an
event) and runs a stand-in for the totals' all-reduce, as bench.py's comm
stream does: --standin sum, a small reduction kernel that uses LDS (torch's
sum over the 3T int64 totals, ~5 us); --standin auto, one VGA frame's
autoDetectHsv (one 1024-lane workgroup for ~40 us: a collective that waits
for its peers holds its CU that long).  Three modes:

  plain     stream A as bench.py creates it;
  reserved  the same, the detector told to leave --reserve CUs free
            (trik_hsv_set_reserved_cus), as bench.py does at N > 1;
  masked    stream A created with a CU mask that leaves --reserve CUs out
            (hipExtStreamCreateWithCUMask): the library sizes the hot kernel's
            grid to the stream's CUs where hipExtStreamGetCUMask reports them
            (stream_cus); the line shows what it reported.

Run under rocprofv3 --kernel-trace; scripts/overlap_trace.py then reports,
for every stand-in launch, whether it started inside a hot-kernel launch or
only after one ended.  Also prints each mode's step time (HIP events)."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))

RANGES = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
          (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]


def masked_stream(torch, reserve):
    """A non-blocking stream on all CUs but the last `reserve` (as a torch
    ExternalStream), the raw handle, and the mask hipExtStreamGetCUMask
    reports for it (popcount)."""
    hip = C.CDLL("libamdhip64.so")
    n = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n + 31) // 32
    mask = (C.c_uint32 * words)()
    for cu in range(n - reserve):
        mask[cu // 32] |= 1 << (cu % 32)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    got = (C.c_uint32 * 32)()
    rc = hip.hipExtStreamGetCUMask(s, C.c_uint32(32), got)
    reported = {"rc": rc, "popcount": sum(bin(v).count("1") for v in got), "words": [hex(v) for v in got[:words + 1]]}
    return torch.cuda.ExternalStream(s.value), s, hip, reported


def run(torch, trik_hsv, mode, reserve, steps, frames_n, standin):
    W, H, T = 640, 480, 4
    ll, fb = 2 * W, H * 2 * W
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    raw = reported = None
    if mode == "masked":
        sa, raw, hip, reported = masked_stream(torch, reserve)
    else:
        sa = torch.cuda.Stream()
    sb = torch.cuda.Stream()
    torch.cuda.set_stream(sa)
    frames = torch.empty(frames_n * fb, dtype=torch.uint8, device="cuda")
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, 0, 0x7A1C, stream=sa)
    det = trik_hsv.Detector()
    if mode == "reserved":
        det.set_reserved_cus(reserve)
    sums = torch.zeros((frames_n, T, 3), dtype=torch.int64, device="cuda")
    tg = torch.zeros((frames_n, T, 4), dtype=torch.int8, device="cuda")
    tot = [torch.zeros((T, 3), dtype=torch.int64, device="cuda") for _ in range(2)]
    red = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in range(2)]
    done = [torch.cuda.Event(), torch.cuda.Event()]
    red_done = [None, None]

    def step(k):
        i = k & 1
        if red_done[i] is not None:
            sa.wait_event(red_done[i])
        det.process_batch_totals(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, RANGES, n_frames=frames_n,
                                 sums=sums, targets=tg, totals=tot[i], stream=sa)
        done[i].record(sa)
        sb.wait_event(done[i])
        with torch.cuda.stream(sb):
            if standin == "sum":  # a small LDS-using reduction on stream B (~5 us)
                red[i].copy_(tot[i].sum())
            else:  # one VGA frame's autoDetectHsv: one 1024-lane workgroup for ~40 us, as a collective
                   # that waits for its peers would hold a CU
                trik_hsv.batch_auto_range(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, n_frames=1, stream=sb)
        if red_done[i] is None:
            red_done[i] = torch.cuda.Event()
        red_done[i].record(sb)

    for k in range(10):
        step(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(sa)
    for k in range(steps):
        step(k)
    sa.wait_stream(sb)
    e1.record(sa)
    torch.cuda.synchronize()
    ok = bool(torch.equal(tot[0], tot[1])) and (standin != "sum" or int(red[0]) == int(tot[0].sum()))
    det.close()
    out = {"mode": mode, "standin": standin, "reserve": reserve if mode != "plain" else 0,
           "ms_per_step": round(e0.elapsed_time(e1) / steps, 4), "steps": steps, "frames": frames_n,
           "totals_ok": ok}
    if reported is not None:
        out["cu_mask_reported"] = reported
        torch.cuda.synchronize()
        hip.hipStreamDestroy(raw)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["plain", "reserved", "masked", "all"], default="all")
    ap.add_argument("--reserve", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--standin", choices=["sum", "auto"], default="sum")
    args = ap.parse_args()
    import torch

    import trik_hsv

    modes = ["plain", "reserved", "masked"] if args.mode == "all" else [args.mode]
    for m in modes:
        print(json.dumps(run(torch, trik_hsv, m, args.reserve, args.steps, args.frames, args.standin)), flush=True)


if __name__ == "__main__":
    main()
