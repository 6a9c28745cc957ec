"""The C ABI's multi-GPU layer (include/trik_hsv.h Layer 3) on the test box's
one GPU: the group (handle + stream + worker thread per device, RCCL
communicator over the devices), the one-process-per-GPU comm, the device
totals kernel, and the C++ host example that drives the group.  Checked
against the CPU oracle.  (Groups of several devices need a multi-GPU node;
their code path per device is the one exercised here.)"""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from gpu_util import BENCH_RANGES, LAYOUT_YUYV

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, LL = 640, 480, 1280
SEED = 0x7A1C


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


def test_device_totals_kernel(torch_dev, hsv):
    torch = torch_dev
    g = torch.Generator().manual_seed(3)
    for n, t in [(0, 1), (1, 4), (333, 3), (4096, 4), (5000, 64)]:
        sums = torch.randint(-2**40, 2**40, (n, t, 3), generator=g, dtype=torch.int64).cuda()
        got = hsv.batch_totals_device(sums)
        torch.cuda.synchronize()
        assert torch.equal(got.cpu(), sums.sum(0).cpu() if n else torch.zeros((t, 3), dtype=torch.int64)), (n, t)


@pytest.mark.parametrize("n_frames", [0, 1, 37, 300])
def test_group_of_one_device(torch_dev, hsv, oracle_mod, n_frames):
    torch = torch_dev
    frames = torch.empty(max(n_frames, 1) * H * LL, dtype=torch.uint8, device="cuda:0")
    if n_frames:
        hsv.synth(frames, W, H, LL, LAYOUT_YUYV, 1, SEED, n_frames=n_frames, first_frame=11)
    torch.cuda.synchronize()
    grp = hsv.Group([0])
    try:
        for _ in range(2):  # the second call reuses the cached tables
            (sums, targets, totals), = grp.process([(frames, n_frames)], W, H, LL, LAYOUT_YUYV, BENCH_RANGES)
            grp.sync()
            host = oracle_mod.synth(max(n_frames, 1), W, H, LL, LAYOUT_YUYV, 1, SEED, first_frame=11)
            want, want_t = oracle_mod.batch(host, H * LL, n_frames, W, H, LL, LAYOUT_YUYV, BENCH_RANGES,
                                            n_threads=16)
            assert np.array_equal(sums.cpu().numpy(), want)
            assert np.array_equal(targets[:, :, :3].cpu().numpy(), want_t)
            assert np.array_equal(totals.cpu().numpy(), want.sum(axis=0) if n_frames else np.zeros((4, 3)))
    finally:
        grp.close()


def test_group_rejects_bad_device_lists(hsv):
    from trik_hsv import _abi

    lib = _abi.load()
    h = C.c_void_p()
    for devs in ([0, 0], [-1], [1 << 20]):
        arr = (C.c_int32 * len(devs))(*devs)
        assert lib.trik_hsv_group_create(len(devs), arr, C.byref(h)) != 0
        assert lib.trik_hsv_last_error()
    assert lib.trik_hsv_group_create(0, None, C.byref(h)) != 0


def test_comm_of_one_rank(torch_dev, hsv):
    """The one-process-per-GPU communicator over a single rank: the totals
    all-reduce is the identity."""
    torch = torch_dev
    from trik_hsv import _abi

    lib = _abi.load()
    torch.cuda.set_device(0)
    uid = (C.c_uint8 * 128)()
    assert lib.trik_hsv_comm_id(uid) == 0, lib.trik_hsv_last_error()
    comm = C.c_void_p()
    assert lib.trik_hsv_comm_create(1, 0, uid, C.byref(comm)) == 0, lib.trik_hsv_last_error()
    try:
        tot = torch.arange(12, dtype=torch.int64, device="cuda").reshape(4, 3) * 1000003
        want = tot.clone()
        s = torch.cuda.current_stream()
        assert lib.trik_hsv_comm_all_reduce_totals(comm, C.c_void_p(tot.data_ptr()), 4,
                                                   C.c_void_p(s.cuda_stream)) == 0
        torch.cuda.synchronize()
        assert torch.equal(tot, want)
        assert lib.trik_hsv_comm_all_reduce_totals(comm, C.c_void_p(tot.data_ptr()), 0, None) != 0
    finally:
        lib.trik_hsv_comm_delete(comm)


def _example():
    exe = os.path.join(ROOT, "examples", "build", "host_multi_gpu")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples"), "multi"], check=True)
    return exe


@pytest.mark.parametrize("total", [0, 64, 4096])
def test_cpp_multi_gpu_host(oracle_mod, total):
    """examples/host_multi_gpu.cpp: a C++ host on the group API; its totals
    agree across devices and with the sum of per-frame sums, and (for a
    sample the CPU checks in seconds) equal the oracle's."""
    r = subprocess.run([_example(), str(total), str(W), str(H), "3"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["ok"] is True and d["frames"] == total
    if total <= 64:
        host = oracle_mod.synth(max(total, 1), W, H, LL, LAYOUT_YUYV, 0, SEED)
        want, _ = oracle_mod.batch(host, H * LL, total, W, H, LL, LAYOUT_YUYV, BENCH_RANGES, n_threads=16)
        assert d["totals"] == want.sum(axis=0).reshape(-1).tolist()
