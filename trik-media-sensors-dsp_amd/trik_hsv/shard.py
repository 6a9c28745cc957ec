"""Multi-GPU plumbing of the path: frame shards and the one collective.

SURVEY section 8(e).  Frames are independent units, so a batch of N frames is
split by frame index into contiguous shards, one per rank (one process per
GPU, torch.distributed over RCCL/xGMI).  Per-frame sums and targets never
leave their rank.  The only exchange is the sum of the per-target batch
totals {points, sumX, sumY} (T x 3 int64, T*24 bytes -- latency-bound, so a
single all-reduce, no bucketing).

The reference has no multi-device path (one DSP, one frame per process call,
trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c:174-264); this is the
batched surface of SURVEY 8(b) spread over ranks.
"""
from __future__ import annotations

from typing import Tuple


def frame_shard(n_frames: int, rank: int, world: int) -> Tuple[int, int]:
    """(first_frame, count) of rank's contiguous share of n_frames.

    Shares differ by at most one frame; every frame belongs to exactly one rank.
    """
    if world <= 0 or not 0 <= rank < world or n_frames < 0:
        raise ValueError(f"bad shard request: n_frames={n_frames} rank={rank} world={world}")
    lo = n_frames * rank // world
    hi = n_frames * (rank + 1) // world
    return lo, hi - lo


def batch_totals(sums):
    """Per-frame sums [F, T, 3] int64 -> per-target batch totals [T, 3] int64."""
    import torch

    if sums.dim() != 3 or sums.shape[-1] != 3 or sums.dtype != torch.int64:
        raise ValueError(f"sums must be [F, T, 3] int64, got {tuple(sums.shape)} {sums.dtype}")
    return torch.sum(sums, dim=0)


def all_reduce_totals(totals, group=None):
    """Sum per-target totals [T, 3] int64 across ranks in place (RCCL for
    device tensors, gloo for host tensors); a no-op without a process group."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
    return totals


def sharded_totals(detector, frames, width, height, line_length, layout, ranges, *,
                   n_frames, frame_stride=None, group=None, stream=None):
    """Run this rank's shard (frames = its frames only, resident on its GPU)
    and return the all-rank per-target totals [T, 3] plus the local per-frame
    sums [n_frames, T, 3]."""
    sums, _ = detector.process_batch(frames, width, height, line_length, layout, ranges,
                                     n_frames=n_frames, frame_stride=frame_stride, stream=stream)
    return all_reduce_totals(batch_totals(sums), group), sums
