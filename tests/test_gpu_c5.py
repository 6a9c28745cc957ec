"""BASELINE config C5 in shape: 32768 VGA YUYV frames sharded over 8 ranks
(4096 frames each, the C3 batch per rank) with the per-target totals
all-reduced -- rehearsed on the test box's one GPU: 8 processes share cuda:0
and reduce over gloo (the driver's scaling run uses RCCL over xGMI, one GPU
per rank).  Each rank runs the bench's full step (trik_hsv_process_batch_totals:
sums, targets and totals in one launch) on its shard.

Checked: the shards tile the 32768 frames; every rank holds the same reduced
totals, equal to the sum of all ranks' per-frame sums; each rank's own totals
equal the sum of its frames' sums; the first, a middle and the last frame of
every shard equal the CPU oracle (sums and targets)."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

W, H, LL = 640, 480, 1280
SEED = 0x7A1C
TOTAL, WORLD = 32768, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist

    import trik_hsv
    from trik_hsv.shard import all_reduce_totals, frame_shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        lo, cnt = frame_shard(TOTAL, rank, world)
        frames = torch.empty(cnt * H * LL, dtype=torch.uint8, device="cuda")
        trik_hsv.synth(frames, W, H, LL, LAYOUT_YUYV, 0, SEED, first_frame=lo, n_frames=cnt)
        det = trik_hsv.Detector()
        T = len(BENCH_RANGES)
        sums = torch.empty((cnt, T, 3), dtype=torch.int64, device="cuda")
        targets = torch.empty((cnt, T, 4), dtype=torch.int8, device="cuda")
        totals = torch.empty((T, 3), dtype=torch.int64, device="cuda")
        det.process_batch_totals(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_frames=cnt, sums=sums,
                                 targets=targets, totals=totals)
        torch.cuda.synchronize()
        own = totals.cpu().clone()
        reduced = all_reduce_totals(totals.cpu())  # gloo reduces host tensors
        kind = det.last_hot_kernel()
        det.close()
        np.save(os.path.join(out_dir, f"sums{rank}.npy"), sums.cpu().numpy())
        np.save(os.path.join(out_dir, f"targets{rank}.npy"), targets.cpu().numpy())
        np.save(os.path.join(out_dir, f"own{rank}.npy"), own.numpy())
        np.save(os.path.join(out_dir, f"reduced{rank}.npy"), reduced.numpy())
        with open(os.path.join(out_dir, f"shard{rank}.json"), "w") as f:
            json.dump([lo, cnt, int(kind)], f)
    finally:
        dist.destroy_process_group()


def test_c5_shape_eight_ranks_on_one_gpu(oracle_mod):
    import torch
    import torch.multiprocessing as mp

    import trik_hsv

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with tempfile.TemporaryDirectory() as out:
        mp.start_processes(_worker, args=(WORLD, _free_port(), out), nprocs=WORLD, join=True, start_method="spawn")
        all_sums, covered = [], []
        for r in range(WORLD):
            with open(os.path.join(out, f"shard{r}.json")) as f:
                lo, cnt, kind = json.load(f)
            assert cnt == TOTAL // WORLD and kind == trik_hsv.HOT_CHROMA, (r, cnt, kind)
            covered.append((lo, cnt))
            s = np.load(os.path.join(out, f"sums{r}.npy"))
            tg = np.load(os.path.join(out, f"targets{r}.npy"))
            assert np.array_equal(np.load(os.path.join(out, f"own{r}.npy")), s.sum(axis=0)), r
            all_sums.append(s)
            # oracle on three frames of the shard
            for i in (0, cnt // 2, cnt - 1):
                host = oracle_mod.synth(1, W, H, LL, LAYOUT_YUYV, 0, SEED, first_frame=lo + i)
                want, _ = oracle_mod.frame(host, W, H, LL, LAYOUT_YUYV, BENCH_RANGES)
                assert np.array_equal(s[i], want), (r, i)
                for t in range(len(BENCH_RANGES)):
                    assert tuple(int(v) for v in tg[i, t, :3]) == oracle_mod.targets(want[t], W, H), (r, i, t)
        assert [lo for lo, _ in covered] == [r * (TOTAL // WORLD) for r in range(WORLD)]
        total = np.concatenate(all_sums).sum(axis=0)
        for r in range(WORLD):
            assert np.array_equal(np.load(os.path.join(out, f"reduced{r}.npy")), total), r
