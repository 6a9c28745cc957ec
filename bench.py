"""Benchmark: HSV-threshold + centroid on batches of 640x480 YUYV frames.

Workload (BASELINE.json configs[2], "C3"): 4096 frames x 640x480 packed YUYV
per GPU, 4 HSV target ranges, frames synthesised on the device (SplitMix64
uniform bytes) before the timed region, so inputs are resident in HBM.  A
step = one full pass of the hot path over the batch: zero the per-frame sums,
the fused detect + reduce kernel, the target epilogue kernel, and the
per-target batch totals (RCCL all-reduce across GPUs when N > 1).

With N GPUs (torch.distributed.run, one process per GPU) each rank owns its
own 4096 frames (global frames rank*4096 ...): weak scaling; at N = 8 this is
BASELINE configs[4] (32768 frames over 8 GPUs).

Prints one JSON line (rank 0).  `roofline` is measured live with HIP events
around the hot kernel on the stream it is launched on; `cpu_baseline` times
the repo's CPU oracle (oracle/, test infrastructure) on a bounded sample of
the same frames on this host's cores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "trik-media-sensors-dsp_amd"))

METRIC = "Mpixels/sec HSV-threshold+centroid on 640×480 YUYV batches; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RANGES = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
          (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]
SEED = 0x7A1C


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 0.7 ms per step: 50 warmup steps bring the clocks to steady state (20
    # steps after 3 warmups read ~10 % slow), 200 timed steps take 0.14 s
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--frames", type=int, default=4096, help="frames per GPU")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--targets", type=int, default=4)
    ap.add_argument("--kind", type=int, default=0, help="0 uniform random bytes, 1 scene")
    ap.add_argument("--cpu-frames", type=int, default=1024, help="CPU baseline sample (frames)")
    ap.add_argument("--cpu-frames-1core", type=int, default=64, help="single-thread CPU sample")
    ap.add_argument("--cpu-frames-emul", type=int, default=32,
                    help="sample of the oracle's intrinsic-level emulation (secondary rate)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hot", choices=["auto", "stripe", "chroma"], default="auto",
                    help="hot kernel (auto = the library's choice: chroma-run for this batch size)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="rocprofv3 FETCH_SIZE summary used for roofline.traffic")
    return ap.parse_args()


def cpu_baseline(args, width, height, ll, n_ranges, gpu_sums):
    """CPU baseline on a bounded sample of the same frames: the clean-room scalar
    restatement of the path (oracle/trik_cpu_baseline.c, a plain CPU port:
    closed-form arithmetic, frames over POSIX threads), checked against the GPU
    sums of those frames.  Threads: this process's CPU share (affinity and
    OMP_NUM_THREADS; 16 per GPU on the bench box) -- the machine's total is
    reported beside it, not used."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    machine = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = machine
    omp = int(os.environ.get("OMP_NUM_THREADS", allowed))
    cores = max(1, min(allowed, omp))
    n = min(args.cpu_frames, args.frames)
    host = oracle.synth(n, width, height, ll, oracle.LAYOUT_YUYV, args.kind, SEED)
    rs = RANGES[:n_ranges]
    t0 = time.perf_counter()
    sums = oracle.cpu_batch(host, height * ll, n, width, height, ll, oracle.LAYOUT_YUYV, rs, n_threads=cores)
    dt = time.perf_counter() - t0
    n1 = min(args.cpu_frames_1core, n)
    t1 = time.perf_counter()
    oracle.cpu_batch(host, height * ll, n1, width, height, ll, oracle.LAYOUT_YUYV, rs, n_threads=1)
    dt1 = time.perf_counter() - t1
    ne = min(args.cpu_frames_emul, n)
    t2 = time.perf_counter()
    emul, _ = oracle.batch(host, height * ll, ne, width, height, ll, oracle.LAYOUT_YUYV, rs, n_threads=cores)
    dt2 = time.perf_counter() - t2
    parity = bool(np.array_equal(sums, gpu_sums[:n])) and bool(np.array_equal(emul, gpu_sums[:ne]))
    px = width * height
    return {"value": round(n * px / dt / 1e6, 3), "unit": "Mpix/s", "cores": cores, "kind": "port",
            "port": "clean-room scalar C restatement (oracle/trik_cpu_baseline.c), POSIX threads",
            "sample": f"{n} frames x {width}x{height} YUYV, {n_ranges} ranges "
                      f"(frames 0..{n - 1} of the GPU batch), {cores} threads, {dt:.2f} s",
            "value_1core": round(n1 * px / dt1 / 1e6, 3),
            "machine_threads": machine, "threads_allowed": allowed,
            "value_intrinsic_emulation": round(ne * px / dt2 / 1e6, 3),
            "cpu_model": cpu_model()}, parity


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(path, bytes_per_launch):
    try:
        with open(path) as f:
            pmc = json.load(f)
        if pmc.get("bytes_per_launch_algorithmic") == bytes_per_launch:
            return pmc.get("hbm_read_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import trik_hsv
    from trik_hsv.shard import all_reduce_totals, batch_totals, frame_shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (not used by the driver): several ranks on one GPU over gloo
    local = int(os.environ.get("TRIK_BENCH_DEVICE", local))
    backend = os.environ.get("TRIK_BENCH_BACKEND", "nccl")  # nccl = RCCL over xGMI
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    W, H, F, T = args.width, args.height, args.frames, args.targets
    ll = 2 * W
    fb = H * ll
    ranges = RANGES[:T]
    frames = torch.empty(F * fb, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    first, count = frame_shard(world * F, rank, world)  # weak scaling: F frames per rank
    assert count == F
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, args.kind, SEED, first_frame=first)
    det = trik_hsv.Detector(hot={"auto": trik_hsv.HOT_AUTO, "stripe": trik_hsv.HOT_STRIPE,
                                 "chroma": trik_hsv.HOT_CHROMA}[args.hot])
    sums = torch.zeros((F, T, 3), dtype=torch.int64, device=dev)

    def step(ev0=None, ev1=None):
        sums.zero_()
        if ev0 is not None:
            ev0.record(stream)
        det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
        if ev1 is not None:
            ev1.record(stream)
        targets = trik_hsv.batch_targets(sums, W, H, stream=stream)
        all_reduce_totals(batch_totals(sums))  # RCCL over xGMI when N > 1: 3*T int64 per step
        return targets

    # cold batch: the first call with this range set compiles the range tables on
    # the host, uploads them and builds the chroma-run tables on the device
    # (stream-ordered, the host does not wait); timed apart from the steps
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sums.zero_()
    torch.cuda.synchronize()
    c0.record(stream)
    h0 = time.perf_counter()
    det.batch_sums(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, ranges, sums, stream=stream)
    host_call_ms = (time.perf_counter() - h0) * 1e3
    c1.record(stream)
    torch.cuda.synchronize()
    cold_ms = c0.elapsed_time(c1)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(*evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    kname = {trik_hsv.HOT_CHROMA: "chroma_kernel", trik_hsv.HOT_STRIPE: "stripe_kernel",
             trik_hsv.HOT_GENERIC: "reduce_kernel"}.get(det.last_hot_kernel(), "?")

    el = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed, kern_ms_max = float(el[0]), float(el[1])

    px_total = world * F * W * H * args.steps
    value = px_total / elapsed / 1e6
    bytes_per_launch = F * fb  # algorithmic: 2 B/pixel read once
    achieved = bytes_per_launch / (kern_ms / 1e3) / 1e9
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Mpix/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: device SplitMix64 uniform bytes, seed 0x7A1C" if args.kind == 0
                else "synthetic: device scene generator (gradients + 6 discs), seed 0x7A1C",
        "config": {"workload": f"C3: batch {F} x {W}x{H} YUYV per GPU, {T} HSV targets"
                               + (f"; {F * world} frames over {world} GPUs" + (" (C5)" if world == 8 else "")
                                  if world > 1 else ""),
                   "frames_per_gpu": F, "width": W, "height": H, "line_length": ll,
                   "targets": T, "layout": "yuyv", "parallelism": f"dp{world} (frame shards)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_traffic(args.pmc, bytes_per_launch),
                     "kernel": f"{kname}<YUYV,{T}>", "kernel_ms": round(kern_ms, 4),
                     "kernel_ms_max_rank": round(kern_ms_max, 4),
                     "bytes_per_launch": bytes_per_launch},
        # first call with a new range set (not in `value`): tables compiled,
        # uploaded and built on the device, then the hot kernel; the host call
        # returns before that work runs
        "cold_batch": {"cold_batch_ms": round(cold_ms, 4), "table_build_ms": round(cold_ms - kern_ms, 4),
                       "host_call_ms": round(host_call_ms, 4)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, parity = cpu_baseline(args, W, H, ll, T, sums.cpu().numpy())
        out["cpu_baseline"] = cb
        out["cpu_sample_parity"] = parity
    if rank == 0:
        print(json.dumps(out), flush=True)
    det.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
