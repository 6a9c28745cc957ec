"""Multi-rank path on CPU: frame shards + the all-reduce of per-target totals.

world_size 2 over gloo on 127.0.0.1 (the driver runs the RCCL/xGMI version of
the same code through bench.py at N = 1, 2, 4, 8).  Each rank synthesises only
its own frames (keyed by global frame index, as bench.py does on the GPU),
computes their per-frame sums with the CPU oracle (the checker), and the
reduced totals must equal a single-process run over the whole batch.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch

from trik_hsv.shard import all_reduce_totals, batch_totals, frame_shard

RANGES = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
          (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]
W, H = 64, 32
SEED = 0x7A1C


@pytest.mark.parametrize("n", [0, 1, 5, 7, 4096])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_frame_shard_partitions_exactly(n, world):
    shards = [frame_shard(n, r, world) for r in range(world)]
    covered = [f for lo, cnt in shards for f in range(lo, lo + cnt)]
    assert covered == list(range(n))
    counts = [cnt for _, cnt in shards]
    assert max(counts) - min(counts) <= 1


def test_frame_shard_rejects_bad_requests():
    for args in [(4, 2, 2), (4, -1, 2), (4, 0, 0), (-1, 0, 1)]:
        with pytest.raises(ValueError):
            frame_shard(*args)


def test_batch_totals_and_single_process_reduce():
    sums = torch.arange(2 * 3 * 3, dtype=torch.int64).reshape(2, 3, 3)
    tot = batch_totals(sums)
    assert tot.tolist() == sums.sum(0).tolist()
    assert all_reduce_totals(tot.clone()).tolist() == tot.tolist()  # no process group: no-op
    with pytest.raises(ValueError):
        batch_totals(sums.to(torch.int32))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_frames, kind, out_dir):
    import torch.distributed as dist

    import oracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        lo, cnt = frame_shard(n_frames, rank, world)
        ll = 2 * W
        frames = oracle.synth(cnt, W, H, ll, oracle.LAYOUT_YUYV, kind, SEED, first_frame=lo)
        sums, _ = oracle.batch(frames, H * ll, cnt, W, H, ll, oracle.LAYOUT_YUYV, RANGES)
        local = torch.from_numpy(sums).reshape(cnt, len(RANGES), 3)
        totals = all_reduce_totals(batch_totals(local))
        # per-frame results stay on their rank; gather them only to check ownership
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, cnt, sums.tolist()))
        if rank == 0:
            np.save(os.path.join(out_dir, "totals.npy"), totals.numpy())
            per_frame = np.zeros((n_frames, len(RANGES), 3), np.int64)
            for g_lo, g_cnt, g_sums in gathered:
                if g_cnt:
                    per_frame[g_lo:g_lo + g_cnt] = np.asarray(g_sums, np.int64)
            np.save(os.path.join(out_dir, "per_frame.npy"), per_frame)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_frames,kind", [(6, 1), (5, 0), (1, 1)])
def test_gloo_world2_totals_match_single_run(oracle_mod, n_frames, kind):
    world = 2
    ll = 2 * W
    with tempfile.TemporaryDirectory() as d:
        torch.multiprocessing.spawn(_worker, args=(world, _free_port(), n_frames, kind, d),
                                    nprocs=world, join=True)
        totals = np.load(os.path.join(d, "totals.npy"))
        per_frame = np.load(os.path.join(d, "per_frame.npy"))
    frames = oracle_mod.synth(n_frames, W, H, ll, oracle_mod.LAYOUT_YUYV, kind, SEED)
    want, _ = oracle_mod.batch(frames, H * ll, n_frames, W, H, ll, oracle_mod.LAYOUT_YUYV, RANGES)
    assert np.array_equal(per_frame, want)
    assert np.array_equal(totals, want.sum(axis=0))
    if kind == 1:
        assert totals[:, 0].sum() > 0  # the scene has target pixels
