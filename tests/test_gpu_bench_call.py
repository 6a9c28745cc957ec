"""The bench's exact call, checked on every frame.

bench.py times trik_hsv_process_batch_totals (the fused step) on C3: 4096
frames of 640x480 YUYV from the device generator (seed 0x7A1C), the 4 bench
ranges, a non-blocking stream and double-buffered totals.  Here the same call
on the same inputs is held to the CPU on all 4096 frames, not a sample:

* every frame's sums against the clean-room scalar CPU port
  (oracle/trik_cpu_baseline.c, held equal to the oracle by
  tests/test_oracle.py::test_cpu_baseline_equals_oracle);
* every frame's targets against the oracle's epilogue (WSEQ:486-505) applied
  to those sums;
* the totals (both buffers) against the CPU sums added over the batch;
* 64 frames spread over the batch against the intrinsic-level oracle itself
  (WSEQ:181-354), sums and targets.

The scene generator (the bench's `scene` line) gets the same treatment.
"""

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

SEED = 0x7A1C
W, H, N = 640, 480, 4096
LL = 2 * W
FB = H * LL
THREADS = 16  # the box's CPU share per GPU
CHUNK = 256   # host frames generated and checked at a time (157 MB)


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def hsv(torch_dev):
    import trik_hsv

    return trik_hsv


def _bench_call(torch, hsv, kind):
    """bench.py's timed call (full_step) twice, into alternating totals buffers."""
    stream = torch.cuda.Stream()
    frames = torch.empty(N * FB, dtype=torch.uint8, device="cuda")
    T = len(BENCH_RANGES)
    with torch.cuda.stream(stream):
        hsv.synth(frames, W, H, LL, LAYOUT_YUYV, kind, SEED, first_frame=0, stream=stream)
        det = hsv.Detector(hot=hsv.HOT_AUTO)
        sums = torch.full((N, T, 3), -7, dtype=torch.int64, device="cuda")
        targets = torch.full((N, T, 4), 99, dtype=torch.int8, device="cuda")
        totals = [torch.full((T, 3), -7, dtype=torch.int64, device="cuda") for _ in range(2)]
        for i in range(4):  # cold (device choice), then fused launches
            det.process_batch_totals(frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_frames=N, frame_stride=FB,
                                     sums=sums, targets=targets, totals=totals[i & 1], stream=stream)
        hot = det.last_hot_kernel()
    stream.synchronize()
    det.close()
    del frames
    return sums.cpu().numpy(), targets.cpu().numpy(), [t.cpu().numpy() for t in totals], hot


@pytest.mark.parametrize("kind", [0, 1], ids=["uniform", "scene"])
def test_bench_call_every_frame(torch_dev, hsv, oracle_mod, kind):
    sums, targets, totals, hot = _bench_call(torch_dev, hsv, kind)
    if kind == 0:
        assert hot == hsv.HOT_CHROMA  # the bench line's kernel
    T = len(BENCH_RANGES)
    want = np.empty_like(sums)
    for lo in range(0, N, CHUNK):
        host = oracle_mod.synth(CHUNK, W, H, LL, LAYOUT_YUYV, kind, SEED, first_frame=lo)
        want[lo:lo + CHUNK] = oracle_mod.cpu_batch(host, FB, CHUNK, W, H, LL, LAYOUT_YUYV, BENCH_RANGES,
                                                   n_threads=THREADS)
        # four frames of every chunk against the intrinsic-level oracle
        pick = np.array([0, CHUNK // 3, 2 * CHUNK // 3, CHUNK - 1])
        sub = host.reshape(CHUNK, FB)[pick].reshape(-1)
        os_, ot = oracle_mod.batch(sub, FB, len(pick), W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_threads=4)
        assert np.array_equal(sums[lo + pick], os_), lo
        assert np.array_equal(targets[lo + pick, :, :3], ot), lo
        del host
    bad = np.nonzero((sums != want).any(axis=(1, 2)))[0]
    assert bad.size == 0, f"frames {bad[:8].tolist()} differ from the CPU port"
    wt = np.empty((N, T, 3), np.int64)
    for f in range(N):
        for t in range(T):
            x, y, z = oracle_mod.targets(want[f, t], W, H)
            wt[f, t] = (x, y, z if z < 128 else z - 256)  # size as int8 bits
    bad = np.nonzero((targets[:, :, :3].astype(np.int64) != wt).any(axis=(1, 2)))[0]
    assert bad.size == 0, f"targets of frames {bad[:8].tolist()} differ from the oracle's epilogue"
    for buf in totals:
        assert np.array_equal(buf, want.sum(0)), "batch totals"
