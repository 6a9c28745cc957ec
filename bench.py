"""Benchmark: HSV-threshold + centroid on batches of 640x480 YUYV frames.

Workload (BASELINE.json configs[2], "C3"): 4096 frames x 640x480 packed YUYV
per GPU, 4 HSV target ranges, frames synthesised on the device (SplitMix64
uniform bytes) before the timed region, so inputs are resident in HBM.  A
step = one full pass of the hot path over the batch
(trik_hsv_process_batch_totals): every frame's sums, its targets (the
epilogue) and the per-target batch totals -- one launch of the chroma-run
kernel at this size (the fused step) -- then the RCCL all-reduce of the totals
across GPUs when N > 1.

Before the warmup (untimed for `value`, reported in their own fields): the
first call of a fresh handle, a batch with a new range set (cold_batch), and
the same step on scene frames (`scene`).

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


# BASELINE.json configs: C3 (the metric's config) and C4 (1280x720, 2 targets)
WORKLOADS = {"c3": dict(frames=4096, width=640, height=480, targets=4),
             "c4": dict(frames=1024, width=1280, height=720, targets=2)}


def workload_name(wl, per_gpu, total, world, w, h, t):
    name = f"{wl.upper()}: batch {per_gpu} x {w}x{h} YUYV per GPU, {t} HSV targets"
    if world > 1:
        c5 = total == 32768 and (w, h, t) == (640, 480, 4)
        name += f"; {total} frames over {world} GPUs" + (" (C5)" if c5 else "")
    return name


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 0.6 ms per step: 200 timed steps take 0.12 s
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                    help="c3 (the headline: 4096 x 640x480, 4 targets) or c4 (1024 x 1280x720, 2 targets)")
    ap.add_argument("--frames", type=int, default=None, help="frames per GPU (default: the workload's)")
    ap.add_argument("--total-frames", type=int, default=None,
                    help="strong scaling: this many frames split over the ranks (C5: 32768)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--targets", type=int, default=None)
    ap.add_argument("--kind", type=int, default=0, help="0 uniform random bytes, 1 scene")
    ap.add_argument("--cpu-frames-all", type=int, default=4096,
                    help="CPU baseline sample on the job's CPUs (the cgroup quota, else every allowed thread)")
    ap.add_argument("--cpu-frames", type=int, default=1024,
                    help="CPU sample on every allowed thread when that exceeds the quota (oversubscribed)")
    ap.add_argument("--scene-launches", type=int, default=60,
                    help="launches timed on scene frames right before the warmup (0: none)")
    ap.add_argument("--cpu-frames-1core", type=int, default=64, help="single-thread CPU sample")
    ap.add_argument("--cpu-frames-emul", type=int, default=32,
                    help="sample of the oracle's intrinsic-level emulation (secondary rate)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--event-every", type=int, default=0,
                    help="bracket every n-th timed step with HIP events for kernel_ms; 0 (default): one event "
                         "pair around the whole timed region when a step is one launch on the stream (the "
                         "fused step at N = 1), else every 4th step (an event record is a stream packet of a "
                         "few us: it delays the launch it brackets)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the cold-batch and scene measurements (PMC passes: only the bench's own launches)")
    ap.add_argument("--hot", choices=["auto", "stripe", "chroma"], default="auto",
                    help="hot kernel (auto = the library's choice: chroma-run for this batch size)")
    ap.add_argument("--collective", choices=["comm", "torch"], default="comm",
                    help="N > 1 over nccl: the totals' all-reduce through the library's own RCCL communicator "
                         "(comm: trik_hsv_comm_all_reduce_totals, double-buffered on a second stream) or "
                         "torch.distributed's (torch: in series on the step's stream)")
    ap.add_argument("--reserve-cus", type=int, default=2,
                    help="with the library's communicator: CUs the hot kernel leaves free so that the all-reduce "
                         "kernel on the second stream runs beside the next step's kernel (trik_hsv_set_reserved_cus; "
                         "the hot kernel takes one 160-KiB-LDS workgroup per CU)")
    ap.add_argument("--comm-self", action="store_true",
                    help="at N = 1 too: a library communicator of one rank, the same double-buffered "
                         "all-reduce (exercises the N > 1 step's code path on one GPU)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="rocprofv3 FETCH_SIZE summary used for roofline.traffic (when measured on these sources)")
    args = ap.parse_args()
    for k, v in WORKLOADS[args.workload].items():
        if getattr(args, k) is None:
            setattr(args, k, v)
    return args


def cpu_baseline(args, width, height, ll, n_ranges, host, gpu_sums):
    """CPU baseline on a bounded sample of the same frames (host: the GPU
    batch's bytes): the clean-room scalar restatement of the path
    (oracle/trik_cpu_baseline.c, a plain CPU port: closed-form arithmetic,
    frames over POSIX threads), checked against the GPU sums of those frames.
    `value` and `cores`: the CPUs this job actually gets -- the cgroup's CPU
    quota when one is set (16 per GPU on the bench box), else every hardware
    thread of the affinity mask.  Beside it: every allowed
    thread when that is more than the quota (time-sliced, labelled
    oversubscribed), one thread, and the oracle's intrinsic-level emulation."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    machine = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = machine
    quota = cgroup_cpus()
    cores = max(1, min(allowed, int(quota))) if quota else allowed
    rs = RANGES[:n_ranges]
    fb = height * ll
    px = width * height

    def run(n, threads):
        t0 = time.perf_counter()
        out = oracle.cpu_batch(host, fb, n, width, height, ll, oracle.LAYOUT_YUYV, rs, n_threads=threads)
        return out, time.perf_counter() - t0

    n_main = min(args.cpu_frames_all, args.frames)
    sums_main, dt_main = run(n_main, cores)
    checks = [(sums_main, n_main)]
    out = {"value": round(n_main * px / dt_main / 1e6, 3), "unit": "Mpix/s", "cores": cores, "kind": "port",
           "port": "clean-room scalar C restatement (oracle/trik_cpu_baseline.c), POSIX threads",
           "sample": f"{n_main} frames x {width}x{height} YUYV, {n_ranges} ranges "
                     f"(frames 0..{n_main - 1} of the GPU batch), {cores} threads, {dt_main:.2f} s",
           "cores_source": ("the cgroup CPU quota" if quota else "the affinity mask (no cgroup quota)")}
    if allowed > cores:  # every allowed thread, beyond the quota: time-sliced
        n_all = min(args.cpu_frames, args.frames)
        sums_all, dt_all = run(n_all, allowed)
        checks.append((sums_all, n_all))
        out["value_all_threads"] = round(n_all * px / dt_all / 1e6, 3)
        out["all_threads"] = allowed
        out["all_threads_note"] = (f"{n_all} frames on all {allowed} allowed threads, {dt_all:.2f} s: "
                                   f"oversubscribed (the job's quota is {quota} CPUs), not the baseline")
    n1 = min(args.cpu_frames_1core, n_main)
    _, dt1 = run(n1, 1)
    ne = min(args.cpu_frames_emul, n_main)
    t2 = time.perf_counter()
    emul, _ = oracle.batch(host, fb, ne, width, height, ll, oracle.LAYOUT_YUYV, rs, n_threads=cores)
    dt2 = time.perf_counter() - t2
    checks.append((emul, ne))
    parity = all(bool(np.array_equal(got, gpu_sums[:n])) for got, n in checks)
    out.update({"value_1core": round(n1 * px / dt1 / 1e6, 3),
                "machine_threads": machine, "threads_allowed": allowed, "cgroup_cpu_quota": quota,
                "value_intrinsic_emulation": round(ne * px / dt2 / 1e6, 3),
                "cpu_model": cpu_model()})
    return out, parity


def cgroup_cpus():
    """The CPU bandwidth quota of this process's cgroup in CPUs (cgroup v2
    cpu.max or v1 cfs quota/period), or None when unlimited/unknown: a box
    that shows 256 hardware threads may grant a GPU job far fewer."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def source_digest():
    """SHA-256 (16 hex) of the library's sources (csrc/ and the public header):
    what a committed PMC pass was measured on (scripts/pmc_summary.py)."""
    import hashlib

    h = hashlib.sha256()
    src = os.path.join(ROOT, "trik-media-sensors-dsp_amd", "csrc")
    for name in sorted(os.listdir(src)):
        if name.endswith((".hip", ".cpp", ".h")):
            with open(os.path.join(src, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    with open(os.path.join(ROOT, "include", "trik_hsv.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def load_traffic(path, bytes_per_launch):
    """(HBM read bytes per launch, where it comes from): the committed PMC pass
    when it was measured at this algorithmic size on these sources, else None."""
    rel = os.path.relpath(path, ROOT)
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None, f"none: {rel} missing"
    if pmc.get("bytes_per_launch_algorithmic") != bytes_per_launch:
        return None, f"none: {rel} was measured at another size"
    if pmc.get("source_digest") != source_digest():
        return None, f"none: {rel} was measured on other sources ({pmc.get('source_digest')})"
    return pmc.get("hbm_read_bytes_per_launch"), (f"committed PMC pass, {rel} (FETCH_SIZE x 2, "
                                                  f"{pmc.get('measured', 'rocprofv3 --pmc')}; same sources)")


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

    W, H, T = args.width, args.height, args.targets
    ll = 2 * W
    fb = H * ll
    ranges = RANGES[:T]
    if args.total_frames:  # strong scaling: a fixed batch split over the ranks
        total = args.total_frames
        first, F = frame_shard(total, rank, world)
    else:  # weak scaling: F frames per rank
        F = args.frames
        total = world * F
        first, count = frame_shard(total, rank, world)
        assert count == F
    # one non-blocking stream for the whole run (torch's default stream is the
    # legacy null stream, whose launches synchronise with every other blocking
    # stream on the device)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    frames = torch.empty(max(F, 1) * fb, dtype=torch.uint8, device=dev)
    trik_hsv.synth(frames, W, H, ll, trik_hsv.LAYOUT_YUYV, args.kind, SEED, first_frame=first)
    hot = {"auto": trik_hsv.HOT_AUTO, "stripe": trik_hsv.HOT_STRIPE, "chroma": trik_hsv.HOT_CHROMA}[args.hot]
    det = trik_hsv.Detector(hot=hot)
    sums = torch.zeros((F, T, 3), dtype=torch.int64, device=dev)
    targets = torch.zeros((F, T, 4), dtype=torch.int8, device=dev)
    # the per-target totals, double-buffered: step k writes buffer k % 2, and
    # its all-reduce (library comm) runs on a second stream while step k + 1's
    # kernel runs; step k + 2 waits (device side) only for that all-reduce
    totals_buf = [torch.zeros((T, 3), dtype=torch.int64, device=dev) for _ in range(2)]
    totals = totals_buf[0]

    # the collective: the library's own communicator when the
    # ranks run over nccl (what a C++ host links), torch.distributed's on
    # request, a host copy over gloo (rehearsal)
    comm = None
    if backend == "nccl" and (world > 1 or args.comm_self) and (args.collective == "comm" or world == 1):
        uid = [trik_hsv.comm_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        comm = trik_hsv.Comm(world, rank, uid[0])
    comm_stream = torch.cuda.Stream(device=dev) if comm is not None else None
    if comm is not None and args.reserve_cus > 0:
        det.set_reserved_cus(args.reserve_cus)
    kern_done = [torch.cuda.Event(), torch.cuda.Event()]
    red_done = [None, None]
    if comm is not None:
        collective = {"call": "trik_hsv_comm_all_reduce_totals (the library's RCCL communicator, C ABI)",
                      "ranks": world, "bytes": 24 * T,
                      "overlap": "double-buffered totals: step k's all-reduce on a second stream while step "
                                 "k+1's kernel runs; step k+2 waits for it on the device",
                      "reserved_cus": args.reserve_cus,
                      "overlap_evidence": "the hot kernel holds one 160-KiB-LDS workgroup on every CU it is given; "
                                          "a kernel on another stream runs beside it on CUs left free (reserved_cus) "
                                          "or takes a CU before the hot workgroup for it starts; rocprofv3 traces: "
                                          "profiles/r06/r06d_overlap_*_trace.txt (scripts/overlap_probe.py)",
                      "tests": "one-rank comm (tests/test_gpu_multirank.py::test_bench_library_comm_one_rank); "
                               "two ranks over nccl: test_bench_two_ranks_library_comm_nccl (runs where 2 GPUs "
                               "are visible)"}
    elif world > 1 and backend == "nccl":
        collective = {"call": "torch.distributed.all_reduce (RCCL)", "ranks": world, "bytes": 24 * T,
                      "overlap": "none: in series after each step's kernel"}
    elif world > 1:
        collective = {"call": f"torch.distributed.all_reduce over {backend} on a host copy (rehearsal)",
                      "ranks": world, "bytes": 24 * T, "overlap": "none"}
    else:
        collective = {"call": "none (one rank)", "ranks": 1}

    def full_step(buf, rs, ev0=None, ev1=None, tot=None):
        """trik_hsv_process_batch_totals: sums, targets and totals of the batch
        (one chroma-run launch where the fused step applies), events around it."""
        if ev0 is not None:
            ev0.record(stream)
        det.process_batch_totals(buf, W, H, ll, trik_hsv.LAYOUT_YUYV, rs, n_frames=F, frame_stride=fb,
                                 sums=sums, targets=targets, totals=totals if tot is None else tot,
                                 stream=stream)
        if ev1 is not None:
            ev1.record(stream)

    nstep = [0]

    def step(ev0=None, ev1=None):
        i = nstep[0] & 1
        nstep[0] += 1
        if comm is not None:
            if red_done[i] is not None:  # the all-reduce that last read this buffer
                stream.wait_event(red_done[i])
            full_step(frames, ranges, ev0, ev1, tot=totals_buf[i])
            kern_done[i].record(stream)
            comm_stream.wait_event(kern_done[i])
            comm.all_reduce_totals(totals_buf[i], stream=comm_stream)
            if red_done[i] is None:
                red_done[i] = torch.cuda.Event()
            red_done[i].record(comm_stream)
            return totals_buf[i]
        full_step(frames, ranges, ev0, ev1)
        if backend == "nccl":
            all_reduce_totals(totals)  # torch.distributed (RCCL) when N > 1: 3*T int64 per step
        elif world > 1:  # gloo rehearsal: reduce a host copy
            totals.copy_(all_reduce_totals(totals.cpu()))
        return totals

    def timed_call(rs):
        """GPU time (HIP events on the stream) and host time of one full step."""
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        c0.record(stream)
        h0 = time.perf_counter()
        full_step(frames, rs)
        host_ms = (time.perf_counter() - h0) * 1e3
        c1.record(stream)
        torch.cuda.synchronize()
        return c0.elapsed_time(c1), host_ms

    # --- untimed for `value`, before the warmup ---------------------------
    # the first call of a fresh handle: table memory allocated, range tables
    # compiled on the host and uploaded, chroma-run tables built on the device
    first_ms, first_host_ms = timed_call(ranges)
    # range sets the handle has not seen, on a warm handle (its table slots
    # already allocated): what a workload that changes ranges pays per change;
    # three new sets, each timed cold and then again (its steady cost), the
    # median difference reported.  After the scene block, so that the clocks
    # are up as in a running workload.  The host call only enqueues.
    def shifted(j):
        return [(r[0] + j if k == 0 else r[0],) + tuple(r[1:]) for k, r in enumerate(ranges)]
    new_ms = new_host_ms = warm_ms = float("nan")
    cold_pairs = []
    if not args.no_extras:
        for j in range(1, 5):  # fill the handle's table slots (4) with other sets
            timed_call(shifted(j))
        for j in (5, 9, 13):  # (hue bounds far enough apart to pack differently)
            c_ms, c_host = timed_call(shifted(j))
            w_ms, _ = timed_call(shifted(j))
            cold_pairs.append((c_ms, w_ms, c_host))
        cold_pairs.sort(key=lambda p: p[0] - p[1])
        new_ms, warm_ms, new_host_ms = cold_pairs[len(cold_pairs) // 2]
        timed_call(ranges)  # back to the bench set (rebuilt)
    full_step(frames, ranges)
    # scene frames: camera-like content, the same step.
    # Last before the warmup, back to back: the timed steps then start from
    # the clocks of a running workload, not from the power controller's
    # transient after the idle gaps above (profiles/r04/r04a_driver_cmd_launches.txt:
    # the same launch ran 478-700 us across those phases)
    scene = None
    if args.scene_launches > 0 and not args.no_extras:
        sframes = torch.empty_like(frames)
        trik_hsv.synth(sframes, W, H, ll, trik_hsv.LAYOUT_YUYV, 1, SEED, first_frame=first)
        full_step(sframes, ranges)
        sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.scene_launches)]
        torch.cuda.synchronize()
        for a, b in sev:
            full_step(sframes, ranges, a, b)
        torch.cuda.synchronize()
        scene_ms = sorted(a.elapsed_time(b) for a, b in sev)
        scene_avg = sum(scene_ms) / len(scene_ms)
        del sframes
        scene = {"kernel_ms": round(scene_avg, 4), "kernel_ms_median": round(scene_ms[len(scene_ms) // 2], 4),
                 "frac": round(F * fb / (scene_avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                 "mpix_per_s": round(F * W * H / (scene_avg / 1e3) / 1e6, 1), "launches": args.scene_launches,
                 "data": "synthetic: device scene generator (gradients + 6 discs), seed 0x7A1C",
                 "note": "the same full step on scene frames, timed back to back right before the warmup "
                         "(not in `value`)"}

    # --- the timed steps ----------------------------------------------------
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # kernel_ms: when a step is exactly one launch on the stream (the fused
    # step on one rank), one event pair around the timed region: the launches'
    # average duration, gaps between them included (an upper bound, and no
    # event packet between launches); otherwise event pairs around every 4th
    # step's launches
    # (one launch: the chroma-run kernel, one group of <= 4 ranges, one rank,
    # no collective on the stream)
    single_launch = det.last_hot_kernel() == trik_hsv.HOT_CHROMA and world == 1 and T <= 4 and comm is None
    every = args.event_every if args.event_every > 0 else (0 if single_launch else 4)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(0, args.steps, every)] if every else []
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    region[0].record(stream)
    last = totals
    for k in range(args.steps):
        if every and k % every == 0:
            last = step(*evs[k // every])
        else:
            last = step()
    if comm is not None:  # the region ends with the last all-reduce
        stream.wait_stream(comm_stream)
    region[1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    region_ms = region[0].elapsed_time(region[1]) / args.steps
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs) if evs else region_ms
    # what the timed steps reduced: the totals after the last step against a
    # fresh sum of this rank's per-frame sums, reduced the same way
    totals = last
    fresh = batch_totals(sums)
    if comm is not None:
        comm.all_reduce_totals(fresh, stream=stream)
        torch.cuda.synchronize()
    elif backend == "nccl":
        all_reduce_totals(fresh)
    elif world > 1:
        fresh = all_reduce_totals(fresh.cpu()).to(dev)
    totals_ok = bool(torch.equal(fresh, totals))
    if comm is not None:  # the other buffer holds the step before's reduction: the same frames
        totals_ok = totals_ok and bool(torch.equal(totals_buf[0], totals_buf[1]))
    ranks = dist.get_world_size() if world > 1 else 1
    kind = det.last_hot_kernel()
    kname = {trik_hsv.HOT_CHROMA: "chroma_kernel", trik_hsv.HOT_STRIPE: "stripe_kernel",
             trik_hsv.HOT_GENERIC: "reduce_kernel", trik_hsv.HOT_MIXED: "mixed"}.get(kind, "?")
    fused = kind == trik_hsv.HOT_CHROMA  # the chroma-run kernel runs the whole step (chroma_fused_ok)

    el = torch.tensor([elapsed, kern_ms, 0.0 if totals_ok else 1.0], dtype=torch.float64, device=dev)
    if world > 1:
        if backend == "nccl":
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        else:
            host = el.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.MAX)
            el.copy_(host)
    elapsed, kern_ms_max = float(el[0]), float(el[1])
    totals_ok = float(el[2]) == 0.0  # on every rank

    px_total = total * W * H * args.steps
    value = px_total / elapsed / 1e6
    bytes_per_launch = F * fb  # algorithmic: 2 B/pixel read once
    achieved = bytes_per_launch / (kern_ms / 1e3) / 1e9
    traffic, traffic_source = load_traffic(args.pmc, bytes_per_launch)
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Mpix/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong" if args.total_frames else "weak", "vs_baseline": None,
        "dtype": "u8", "ranks": ranks, "backend": (("nccl (RCCL)" if backend == "nccl" else backend)
                                                  if world > 1 else "none (one process)"),
        "collective": collective,
        "totals_check": {"ok": totals_ok, "frames_reduced": total,
                         "points": [int(x) for x in totals[:, 0].tolist()],
                         "how": "after the timed steps, a fresh sum of the rank's per-frame sums, "
                                "all-reduced over the same backend, equals the totals the steps reduced"},
        "data": "synthetic: device SplitMix64 uniform bytes, seed 0x7A1C" if args.kind == 0
                else "synthetic: device scene generator (gradients + 6 discs), seed 0x7A1C",
        "config": {"workload": workload_name(args.workload, F, total, world, W, H, T),
                   "frames_per_gpu": F, "frames_total": total, "width": W, "height": H, "line_length": ll,
                   "targets": T, "layout": "yuyv", "parallelism": f"dp{world} (frame shards)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_source,
                     "kernel": f"{kname}<YUYV,{T}>", "kernel_ms": round(kern_ms, 4),
                     "kernel_ms_max_rank": round(kern_ms_max, 4),
                     "kernel_ms_how": ("one event pair around the timed region / steps (each step is this one "
                                       "launch plus the library's stream mark and, every 8th call, its 8-byte "
                                       "AUTO probe readback; the gaps between launches included)" if not evs else
                                       f"event pairs around every {every}-th step's launches ({len(evs)} steps)"),
                     "region_ms_per_step": round(region_ms, 4),
                     "kernel_scope": ("the step's one launch (fused: its frames' sums zeroed and added, targets and totals written "
                                      "by the same kernel)" if fused else
                                      "the step's launches (zero the sums, hot kernel, epilogue, totals)"),
                     "bytes_per_launch": bytes_per_launch},
    }
    if not args.no_extras:
        out["cold_batch"] = {"cold_batch_ms": round(new_ms, 4), "table_build_ms": round(new_ms - warm_ms, 4),
                       "warm_same_set_ms": round(warm_ms, 4),
                       "host_call_ms": round(new_host_ms, 4),
                       "first_call_ms": round(first_ms, 4), "first_call_host_ms": round(first_host_ms, 4),
                       "sets_ms": [[round(c, 4), round(w, 4)] for c, w, _ in cold_pairs],
                       "note": "cold_batch_ms: one step with a range set new to a warm handle (tables "
                               "compiled and built on the device, then the hot kernel); "
                               "table_build_ms = cold_batch_ms - the same set's next step, the median "
                               "over three new sets (sets_ms: [cold, next] each); first_call: a fresh "
                               "handle, table memory allocated too; measured before the scene block and "
                               "the warmup"}
    if scene is not None:
        out["scene"] = scene
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n_host = min(F, max(args.cpu_frames_all, args.cpu_frames))
        host = frames[: n_host * fb].cpu().numpy()
        cb, parity = cpu_baseline(args, W, H, ll, T, host, sums.cpu().numpy())
        out["cpu_baseline"] = cb
        out["cpu_sample_parity"] = parity
    if rank == 0:
        print(json.dumps(out), flush=True)
    det.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
