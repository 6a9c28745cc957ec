"""Full-size batches of the two single-GPU configs, checked against the CPU.

C3 (the bench workload): 4096 x 640x480 YUYV, 4 ranges.  C4: 1024 x 1280x720
YUYV, 2 ranges.  Both run through the C ABI with the library's AUTO choice
(the chroma-run kernel at these sizes).  The checkers:

* the oracle (oracle/trik_oracle.c, the intrinsic-level restatement of
  WSEQ:181-354) on a sample of frames spread over the batch;
* the clean-room scalar CPU port (oracle/trik_cpu_baseline.c, held equal to
  the oracle by tests/test_oracle.py::test_cpu_baseline_equals_oracle) on many
  more frames -- it is ~10x faster than the intrinsic emulation;
* the target epilogue of every checked frame against the oracle's.
"""

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

SEED = 0x7A1C
THREADS = 16  # the box's CPU share per GPU


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


def _host_frames(oracle_mod, idx, w, h, ll, kind=0):
    """The synthetic frames with global indices idx (same generator as the device)."""
    out = np.empty((len(idx), h * ll), np.uint8)
    for k, f in enumerate(idx):
        out[k] = oracle_mod.synth(1, w, h, ll, LAYOUT_YUYV, kind, SEED, first_frame=int(f)).reshape(-1)
    return out.reshape(-1)


def _run_full(torch, hsv, n, w, h, ranges, kind=0):
    ll = 2 * w
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, kind, SEED)
    det = hsv.Detector()
    s1, t1 = det.process_batch(dev, w, h, ll, LAYOUT_YUYV, ranges)
    s2, t2 = det.process_batch(dev, w, h, ll, LAYOUT_YUYV, ranges)
    hot = det.last_hot_kernel()
    det.close()
    torch.cuda.synchronize()
    assert torch.equal(s1, s2) and torch.equal(t1, t2), "not deterministic across runs"
    del dev
    return s1.cpu().numpy(), t1.cpu().numpy(), hot


def _check(oracle_mod, sums, targets, idx_oracle, idx_cpu, w, h, ranges, kind=0):
    ll = 2 * w
    host = _host_frames(oracle_mod, idx_oracle, w, h, ll, kind)
    want, want_t = oracle_mod.batch(host, h * ll, len(idx_oracle), w, h, ll, LAYOUT_YUYV, ranges,
                                    n_threads=THREADS)
    assert np.array_equal(sums[idx_oracle], want)
    assert np.array_equal(targets[idx_oracle, :, :3], want_t)
    for lo in range(0, len(idx_cpu), 256):  # bounded host memory
        part = idx_cpu[lo:lo + 256]
        host = _host_frames(oracle_mod, part, w, h, ll, kind)
        got = oracle_mod.cpu_batch(host, h * ll, len(part), w, h, ll, LAYOUT_YUYV, ranges, n_threads=THREADS)
        bad = np.nonzero((got != sums[part]).any(axis=(1, 2)))[0]
        assert bad.size == 0, f"frames {part[bad[:8]].tolist()} differ from the CPU port"


def test_c3_full_batch(torch_dev, hsv, oracle_mod):
    """4096 x 640x480, T=4: every 8th frame (512) against the CPU port, 32 of
    them against the oracle, targets included."""
    w, h, n = 640, 480, 4096
    sums, targets, hot = _run_full(torch_dev, hsv, n, w, h, BENCH_RANGES)
    assert hot == hsv.HOT_CHROMA
    _check(oracle_mod, sums, targets, np.arange(0, n, 128), np.arange(0, n, 8), w, h, BENCH_RANGES)
    assert sums[:, :, 0].min() > 0  # uniform data hits every range in every frame


def test_c4_full_batch(torch_dev, hsv, oracle_mod):
    """1024 x 1280x720, T=2 (BASELINE configs C4): every frame against the CPU
    port, every 16th (64 frames) against the oracle, targets included."""
    w, h, n = 1280, 720, 1024
    ranges = BENCH_RANGES[:2]
    sums, targets, hot = _run_full(torch_dev, hsv, n, w, h, ranges)
    assert hot == hsv.HOT_CHROMA
    _check(oracle_mod, sums, targets, np.arange(0, n, 16), np.arange(n), w, h, ranges)


def test_c4_scene_batch(torch_dev, hsv, oracle_mod):
    """C4 geometry on the scene generator (long chroma runs, camera-like)."""
    w, h, n = 1280, 720, 256
    ranges = BENCH_RANGES[:2]
    sums, targets, _ = _run_full(torch_dev, hsv, n, w, h, ranges, kind=1)
    _check(oracle_mod, sums, targets, np.arange(0, n, 32), np.arange(n), w, h, ranges, kind=1)
