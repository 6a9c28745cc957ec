"""The HIP path under several ranks (one process per rank, frame shards, the
all-reduce of per-target totals), rehearsed on the one GPU of the test box.

The driver runs the RCCL/xGMI form on an 8-GPU node (bench.py at N = 1, 2, 4,
8); here two processes share cuda:0 and reduce over gloo, which runs the same
product code (trik_hsv.shard + the C ABI) per rank.  Checked against the CPU
oracle: every rank's per-frame sums, and the reduced totals equal the totals
of the whole batch.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, LL = 640, 480, 1280
SEED = 0x7A1C


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_frames, hot, out_dir):
    import torch
    import torch.distributed as dist

    import trik_hsv
    from trik_hsv.shard import all_reduce_totals, batch_totals, frame_shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        lo, cnt = frame_shard(n_frames, rank, world)
        frames = torch.empty(max(cnt, 1) * H * LL, dtype=torch.uint8, device="cuda")
        trik_hsv.synth(frames, W, H, LL, LAYOUT_YUYV, 0, SEED, first_frame=lo, n_frames=cnt)
        det = trik_hsv.Detector(hot=hot)
        sums, _ = det.process_batch(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_frames=cnt)
        totals = all_reduce_totals(batch_totals(sums).cpu())  # gloo reduces host tensors
        det.close()
        np.save(os.path.join(out_dir, f"sums{rank}.npy"), sums.cpu().numpy())
        np.save(os.path.join(out_dir, f"totals{rank}.npy"), totals.numpy())
        with open(os.path.join(out_dir, f"shard{rank}.json"), "w") as f:
            json.dump([lo, cnt], f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_frames,hot", [(40, "auto"), (33, "chroma")])
def test_two_ranks_on_one_gpu(n_frames, hot, oracle_mod):
    import torch
    import torch.multiprocessing as mp

    import trik_hsv

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    hot_id = {"auto": trik_hsv.HOT_AUTO, "chroma": trik_hsv.HOT_CHROMA}[hot]
    world = 2
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(world, _free_port(), n_frames, hot_id, out), nprocs=world,
                           join=True, start_method="spawn")
        host = oracle_mod.synth(n_frames, W, H, LL, LAYOUT_YUYV, 0, SEED)
        want, _ = oracle_mod.batch(host, H * LL, n_frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_threads=16)
        covered = []
        for r in range(world):
            with open(os.path.join(out, f"shard{r}.json")) as f:
                lo, cnt = json.load(f)
            covered += list(range(lo, lo + cnt))
            assert np.array_equal(np.load(os.path.join(out, f"sums{r}.npy")), want[lo:lo + cnt]), r
            assert np.array_equal(np.load(os.path.join(out, f"totals{r}.npy")), want.sum(axis=0)), r
        assert covered == list(range(n_frames))


@pytest.mark.parametrize("extra", [["--frames", "64"], ["--total-frames", "97"]])
def test_bench_two_ranks_rehearsal(extra):
    """bench.py's N > 1 path (barriers, max-over-ranks timing, the all-reduce)
    with two ranks on cuda:0 over gloo: one JSON line from rank 0."""
    env = dict(os.environ, TRIK_BENCH_BACKEND="gloo", TRIK_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    # the line proves what it measured: the process group's size, its backend,
    # and the reduced totals equal to a fresh reduction of the per-frame sums
    assert d["ranks"] == 2 and d["backend"] == "gloo"
    assert d["collective"]["ranks"] == 2 and "gloo" in d["collective"]["call"]
    chk = d["totals_check"]
    assert chk["ok"] is True and chk["frames_reduced"] == d["config"]["frames_total"]
    assert len(chk["points"]) == d["config"]["targets"] and all(p > 0 for p in chk["points"])
    if "--total-frames" in extra:
        assert d["scaling"] == "strong" and d["config"]["frames_total"] == 97
    else:
        assert d["scaling"] == "weak" and d["config"]["frames_total"] == 128


def test_bench_library_comm_one_rank():
    """bench.py's N > 1 collective path on one GPU (--comm-self): the totals
    all-reduced through the library's own communicator
    (trik_hsv_comm_all_reduce_totals, a comm of one rank), double-buffered on a
    second stream; the line names the call and its totals check holds."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "6", "--warmup", "3", "--frames", "64",
           "--no-cpu-baseline", "--no-extras", "--comm-self"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["collective"]["call"].startswith("trik_hsv_comm_all_reduce_totals")
    assert "double-buffered" in d["collective"]["overlap"]
    chk = d["totals_check"]
    assert chk["ok"] is True and chk["frames_reduced"] == 64 and all(p > 0 for p in chk["points"])


def test_bench_two_ranks_library_comm_nccl():
    """bench.py's multi-GPU collective as the driver runs it: two ranks, one
    GPU each, over nccl (RCCL), the totals all-reduced by the library's own
    communicator, double-buffered on a second stream -- buffer reuse two steps
    apart, the red_done waits and the two buffers' equality across ranks are
    all inside totals_check.  Needs two visible GPUs (the test box has one:
    skipped there; the driver's 8-GPU SCALE run is the same code path)."""
    import torch

    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("TRIK_BENCH_BACKEND", None)
    env.pop("TRIK_BENCH_DEVICE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "3", "--frames", "64",
           "--no-cpu-baseline", "--no-extras"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and d["backend"].startswith("nccl")
    assert d["collective"]["call"].startswith("trik_hsv_comm_all_reduce_totals") and d["collective"]["ranks"] == 2
    chk = d["totals_check"]
    assert chk["ok"] is True and chk["frames_reduced"] == 128 and all(p > 0 for p in chk["points"])
