"""Host-side behaviour of the batched API around the device tables
(trik_hsv_abi.cpp: acquire_tables, ensure_chroma, plan_hot, StreamUses):

* the first call with a new range set enqueues the table build and the hot
  kernels without waiting on the host (the device picks the kernel by the
  builder's cost while the share is unknown);
* one handle used from two streams, with the same and with different range
  sets, gives the oracle's sums (each stream waits for the uploads it reads,
  and a new range set never overwrites tables a queued kernel still reads);
* buffers that are not device memory are rejected by the C ABI.
"""
import ctypes as C
import time

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV, T0, T1

pytestmark = pytest.mark.gpu


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


def _busy(torch, ms=150.0):
    """Keep the current stream busy for about `ms` (a device-side spin)."""
    torch.cuda._sleep(int(ms * 1e-3 * 1.0e9))


def test_new_range_set_does_not_block(torch_dev, hsv, oracle_mod):
    torch = torch_dev
    w, h, ll, n = 640, 480, 1280, 32  # TRIK_HSV_CHROMA_MIN_PIXELS: the chroma path
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C, first_frame=5)
    host = dev.cpu().numpy()
    d = hsv.Detector()
    try:
        s = torch.cuda.current_stream()
        for ranges in (BENCH_RANGES, [T0, T1]):  # both new to the handle
            sums = torch.zeros((n, len(ranges), 3), dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            t_spin = time.perf_counter()
            _busy(torch)
            t0 = time.perf_counter()
            d.batch_sums(dev, w, h, ll, LAYOUT_YUYV, ranges, sums)
            dt = time.perf_counter() - t0
            pending = not s.query()
            torch.cuda.synchronize()
            spin = time.perf_counter() - t_spin
            assert spin > 0.05, "the spin kernel did not keep the stream busy"
            assert pending and dt < 0.5 * spin, (dt, spin)
            want, _ = oracle_mod.batch(host, h * ll, n, w, h, ll, LAYOUT_YUYV, ranges, n_threads=8)
            assert np.array_equal(sums.cpu().numpy(), want)
            assert d.last_hot_kernel() == hsv.HOT_CHROMA
    finally:
        d.close()


def test_one_handle_two_streams(torch_dev, hsv, oracle_mod):
    torch = torch_dev
    w, h, ll, n = 640, 480, 1280, 32
    dev = torch.empty(n * h * ll, dtype=torch.uint8, device="cuda")
    hsv.synth(dev, w, h, ll, LAYOUT_YUYV, 0, 0x7A1C, first_frame=77)
    host = dev.cpu().numpy()
    sets = [BENCH_RANGES, [T0], [T1, T0], BENCH_RANGES[1:], [(10, 350, 0, 100, 0, 100)], [T0]]
    want = [oracle_mod.batch(host, h * ll, n, w, h, ll, LAYOUT_YUYV, r, n_threads=8)[0] for r in sets]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    d = hsv.Detector()
    try:
        for rep in range(2):
            outs = []
            for i, ranges in enumerate(sets):
                st = sa if i % 2 == 0 else sb
                with torch.cuda.stream(st):
                    if i % 3 == 0:
                        _busy(torch, 20.0)  # let the two streams overlap
                    sums = torch.zeros((n, len(ranges), 3), dtype=torch.int64, device="cuda")
                    d.batch_sums(dev, w, h, ll, LAYOUT_YUYV, ranges, sums, stream=st)
                    outs.append(sums)
            torch.cuda.synchronize()
            for i, (got, exp) in enumerate(zip(outs, want)):
                assert np.array_equal(got.cpu().numpy(), exp), (rep, i, sets[i])
    finally:
        d.close()


def test_host_frames_rejected(torch_dev, hsv):
    from trik_hsv import _abi

    torch = torch_dev
    lib = _abi.load()
    d = hsv.Detector()
    try:
        host = np.zeros(2 * 480 * 1280, np.uint8)
        b = _abi.FrameBatch(host.ctypes.data, 480 * 1280, 2, 640, 480, 1280, LAYOUT_YUYV)
        arr = (_abi.InArgsAlg * 1)(_abi.InArgsAlg(*T0, 0))
        sums = torch.zeros((2, 1, 3), dtype=torch.int64, device="cuda")
        rc = lib.trik_hsv_batch_sums(d._h, C.byref(b), arr, 1, C.c_void_p(sums.data_ptr()), None)
        assert rc != 0 and b"device" in lib.trik_hsv_last_error()
    finally:
        d.close()
