"""trik_hsv -- host-side mirror of the TRIK object-sensor operator, MI355X-native.

Everything computes in libtrik_hsv.so (HIP kernels for gfx950 + the C++
XDAIS-shaped layer) through its C ABI (include/trik_hsv.h).  PyTorch is used
only to own device memory and streams.  There is no CPU fallback.

Two surfaces, mirroring the reference (paths relative to the reference checkout):
  * ObjectSensor -- the codec instance: create / control / process / delete of
    trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c, one host frame per
    process() call, OutArgs.targetX/targetY/targetSize out.
  * Detector -- the batched device path: N frames resident in HBM, T HSV
    ranges, per-frame per-range {points, sumX, sumY} and targets.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Sequence, Tuple

from . import _abi
from ._abi import (FORMAT_RGB565X, FORMAT_UNKNOWN, FORMAT_YUV422, FORMAT_YUV422P,  # noqa: F401
                   IALG_EFAIL, IALG_EOK, IVIDTRANSCODE_EFAIL, IVIDTRANSCODE_EOK,
                   IVIDTRANSCODE_EUNSUPPORTED, LAYOUT_OV7670, LAYOUT_YUYV, XDM_FLUSH,
                   XDM_GETBUFINFO, XDM_GETSTATUS, XDM_GETVERSION, XDM_RESET, XDM_SETDEFAULT,
                   XDM_SETPARAMS)

_lib = _abi.load()  # fails loudly when the native library is missing

Range = Tuple[int, int, int, int, int, int]  # hue_from, hue_to, sat_from, sat_to, val_from, val_to


class TrikHsvError(RuntimeError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what} failed (rc={rc}): {_abi.last_error()}")
        self.rc = rc


def version() -> str:
    return _lib.trik_hsv_version().decode()


def _ranges(ranges: Iterable[Sequence[int]]):
    rs = [tuple(int(v) for v in r) for r in ranges]
    arr = (_abi.InArgsAlg * max(1, len(rs)))()
    for i, r in enumerate(rs):
        arr[i] = _abi.InArgsAlg(*r[:6], 0)
    return arr, len(rs)


def frame_bytes(width: int, height: int, line_length: int, layout: int) -> int:
    return height * line_length * (2 if layout == LAYOUT_OV7670 else 1)


def _stream_ptr(stream, tensor) -> C.c_void_p:
    """`stream`, or torch's current stream of the device `tensor` lives on."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream(tensor.device)
    return C.c_void_p(s.cuda_stream)


def _batch(frames, width, height, line_length, layout, n_frames=None, frame_stride=None):
    fb = frame_bytes(width, height, line_length, layout)
    if frame_stride is None:
        frame_stride = fb
    if n_frames is None:
        n_frames = frames.numel() // frame_stride if frame_stride else 0
    if frames.dtype.itemsize != 1 or not frames.is_cuda:
        raise ValueError("frames must be a uint8 CUDA (HIP) tensor")
    if n_frames > 0 and (n_frames - 1) * frame_stride + fb > frames.numel():
        raise ValueError("frames tensor too small for the batch geometry")
    return _abi.FrameBatch(frames.data_ptr(), frame_stride, n_frames, width, height, line_length,
                           layout)


HOT_AUTO, HOT_STRIPE, HOT_CHROMA, HOT_GENERIC = 0, 1, 2, 3
HOT_MIXED = 4  # last_hot_kernel(): the call's groups of 4 ranges ran different kernels


class _HotKernel:
    """Hot-kernel selection of one handle (trik_hsv_set_hot_kernel)."""

    def set_hot_kernel(self, kind: int) -> int:
        """HOT_AUTO (the chroma-run kernel for large batches), HOT_STRIPE,
        HOT_CHROMA or HOT_GENERIC for this handle's batched sums.  Returns the
        previous setting.  Results are identical."""
        prev = _lib.trik_hsv_set_hot_kernel(self._h, int(kind))
        if prev < 0:
            raise ValueError(f"unknown hot kernel {kind}")
        return prev

    def last_hot_kernel(self) -> int:
        """The kernel this handle's last hot launch ran."""
        return _lib.trik_hsv_last_hot_kernel(self._h)

    def set_reserved_cus(self, n: int) -> int:
        """CUs the chroma-run kernel leaves free for kernels on other streams
        (trik_hsv_set_reserved_cus).  Returns the previous setting."""
        prev = _lib.trik_hsv_set_reserved_cus(self._h, int(n))
        if prev < 0:
            raise ValueError(f"reserved CUs out of range: {n}")
        return prev


class Detector(_HotKernel):
    """Batched HSV-threshold + centroid over frames resident in device memory.

    Owns one library handle, bound to `device` (default: the current device;
    device tables are compiled per range set and cached).  Methods enqueue on
    `stream` (default: torch's current stream of the frames' device) and do
    not synchronise.
    """

    def __init__(self, device=None, hot: int = HOT_AUTO):
        import torch

        h = C.c_void_p()
        p = _default_params(0)
        with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
            rc = _lib.TRIK_VIDTRANSCODE_CV_create(C.byref(p), C.byref(h))
        if rc != IALG_EOK:
            raise TrikHsvError(rc, "TRIK_VIDTRANSCODE_CV_create")
        self._h = h
        if hot != HOT_AUTO:
            self.set_hot_kernel(hot)

    def close(self):
        if getattr(self, "_h", None):
            _lib.TRIK_VIDTRANSCODE_CV_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process_batch(self, frames, width, height, line_length, layout, ranges, *, n_frames=None,
                      frame_stride=None, stream=None, sums=None, targets=None):
        """Returns (sums int64 [N,T,3] = points/sumX/sumY, targets int8 [N,T,4] = x/y/size/0)."""
        import torch

        b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
        arr, T = _ranges(ranges)
        if sums is None:
            sums = torch.empty((b.n_frames, T, 3), dtype=torch.int64, device=frames.device)
        if targets is None:
            targets = torch.empty((b.n_frames, T, 4), dtype=torch.int8, device=frames.device)
        rc = _lib.trik_hsv_process_batch(self._h, C.byref(b), arr, T, C.c_void_p(sums.data_ptr()),
                                         C.c_void_p(targets.data_ptr()), _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_process_batch")
        return sums, targets

    def process_batch_totals(self, frames, width, height, line_length, layout, ranges, *, n_frames=None,
                             frame_stride=None, stream=None, sums=None, targets=None, totals=None):
        """The full step (trik_hsv_process_batch_totals): sums, targets and the
        per-target batch totals; one launch per group of 4 ranges where the
        chroma-run kernel runs on >= 4 frames per CU.  Returns (sums, targets,
        totals int64 [T,3])."""
        import torch

        b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
        arr, T = _ranges(ranges)
        if sums is None:
            sums = torch.empty((b.n_frames, T, 3), dtype=torch.int64, device=frames.device)
        if targets is None:
            targets = torch.empty((b.n_frames, T, 4), dtype=torch.int8, device=frames.device)
        if totals is None:
            totals = torch.empty((T, 3), dtype=torch.int64, device=frames.device)
        rc = _lib.trik_hsv_process_batch_totals(self._h, C.byref(b), arr, T, C.c_void_p(sums.data_ptr()),
                                                C.c_void_p(targets.data_ptr()), C.c_void_p(totals.data_ptr()),
                                                _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_process_batch_totals")
        return sums, targets, totals

    def batch_sums(self, frames, width, height, line_length, layout, ranges, sums, *,
                   n_frames=None, frame_stride=None, stream=None):
        """Hot kernel only; ADDS into `sums` (int64 [N,T,3], caller zeroes it)."""
        b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
        arr, T = _ranges(ranges)
        rc = _lib.trik_hsv_batch_sums(self._h, C.byref(b), arr, T, C.c_void_p(sums.data_ptr()),
                                      _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_batch_sums")
        return sums

    def chroma_flagged_share(self) -> float:
        """The chroma-run kernel's expected exact-path word share for the
        current batched-sums range set (-1 before its tables are built)."""
        v = C.c_double()
        rc = _lib.trik_hsv_chroma_share(self._h, C.byref(v))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_chroma_share")
        return v.value

    def chroma_measured_share(self) -> float:
        """The exact-path word share the chroma-run kernel measured on this
        handle's recent AUTO batches of the current range set (-1 unknown)."""
        v = C.c_double()
        rc = _lib.trik_hsv_chroma_measured_share(self._h, C.byref(v))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_chroma_measured_share")
        return v.value

    def batch_masks(self, frames, width, height, line_length, layout, ranges, *, n_frames=None,
                    frame_stride=None, stream=None):
        """Verification mode: returns (masks uint8 [N,H,W], sums int64 [N,T,3])."""
        import torch

        b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
        arr, T = _ranges(ranges)
        masks = torch.zeros((b.n_frames, height, width), dtype=torch.uint8, device=frames.device)
        sums = torch.zeros((b.n_frames, T, 3), dtype=torch.int64, device=frames.device)
        rc = _lib.trik_hsv_batch_masks(self._h, C.byref(b), arr, T, C.c_void_p(masks.data_ptr()),
                                       C.c_void_p(sums.data_ptr()), _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_batch_masks")
        return masks, sums

    def batch_preview(self, frames, width, height, line_length, layout, hsv_range, sums, *,
                      out_width=None, out_height=None, out_line_length=None, n_frames=None,
                      frame_stride=None, sums_pitch=1, stream=None):
        """RGB565X previews (uint8 [N, out_height, out_line_length]) for one range;
        `sums` holds that range's per-frame sums (every `sums_pitch` entries)."""
        import torch

        b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
        ow = width // 2 if out_width is None else out_width
        oh = height // 2 if out_height is None else out_height
        oll = 2 * ow if out_line_length is None else out_line_length
        previews = torch.empty((b.n_frames, oh, oll), dtype=torch.uint8, device=frames.device)
        arr, _ = _ranges([hsv_range])
        rc = _lib.trik_hsv_batch_preview(self._h, C.byref(b), arr, C.c_void_p(sums.data_ptr()),
                                         sums_pitch, ow, oh, oll, C.c_void_p(previews.data_ptr()),
                                         oh * oll, _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_batch_preview")
        return previews


    def blob_batch(self, frames, width, height, line_length, hsv, *, n_frames=None, frame_stride=None,
                   meta=False, labels=False, stream=None):
        """The ov7670 multi-blob sensor over N frames (OSEQ:516-602) for the range
        hsv = (hue, hueTol, sat, satTol, val, valTol).  Returns a dict of device
        tensors: targets int8 [N, 8, 4] (x, y, size, 0), top int32 [N, 8, 3]
        (size, sum_x, sum_y), n_labels int32 [N], and meta uint8 / labels int16
        [N, H/4, W/4] when asked (else meta is the handle's scratch, None here)."""
        import torch

        b = _batch(frames, width, height, line_length, LAYOUT_OV7670, n_frames, frame_stride)
        dev = frames.device
        out = {"targets": torch.empty((b.n_frames, 8, 4), dtype=torch.int8, device=dev),
               "top": torch.empty((b.n_frames, 8, 3), dtype=torch.int32, device=dev),
               "n_labels": torch.empty((b.n_frames,), dtype=torch.int32, device=dev),
               "meta": torch.empty((b.n_frames, height // 4, width // 4), dtype=torch.uint8, device=dev)
               if meta else None,
               "labels": torch.empty((b.n_frames, height // 4, width // 4), dtype=torch.int16, device=dev)
               if labels else None}
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        alg = _abi.OV7670InArgsAlg(1, *[int(v) for v in hsv], 0)
        rc = _lib.trik_hsv_blob_batch(self._h, C.byref(b), C.byref(alg), ptr(out["targets"]), ptr(out["top"]),
                                      ptr(out["meta"]), ptr(out["labels"]), ptr(out["n_labels"]),
                                      _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_blob_batch")
        return out

    def blob_preview(self, frames, width, height, line_length, meta, top, *, out_width=None,
                     out_height=None, out_line_length=None, n_frames=None, frame_stride=None, stream=None):
        """Multi-blob previews (uint8 [N, out_height, out_line_length]) from blob_batch's meta and top."""
        import torch

        b = _batch(frames, width, height, line_length, LAYOUT_OV7670, n_frames, frame_stride)
        ow = width // 2 if out_width is None else out_width
        oh = height // 2 if out_height is None else out_height
        oll = 2 * ow if out_line_length is None else out_line_length
        previews = torch.empty((b.n_frames, oh, oll), dtype=torch.uint8, device=frames.device)
        rc = _lib.trik_hsv_blob_preview(self._h, C.byref(b), C.c_void_p(meta.data_ptr()),
                                        C.c_void_p(top.data_ptr()), ow, oh, oll,
                                        C.c_void_p(previews.data_ptr()), oh * oll, _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_blob_preview")
        return previews

    def line_preview(self, frames, width, height, line_length, val_from, val_to, sums, *,
                     out_width=None, out_height=None, out_line_length=None, n_frames=None,
                     frame_stride=None, stream=None):
        """Line-sensor previews (uint8 [N, out_height, out_line_length]) from the
        per-frame sums of line_batch (LSEQ:283-291, 433-467)."""
        import torch

        b = _batch(frames, width, height, line_length, LAYOUT_OV7670, n_frames, frame_stride)
        ow = width // 2 if out_width is None else out_width
        oh = height // 2 if out_height is None else out_height
        oll = 2 * ow if out_line_length is None else out_line_length
        previews = torch.empty((b.n_frames, oh, oll), dtype=torch.uint8, device=frames.device)
        rc = _lib.trik_hsv_line_preview(self._h, C.byref(b), int(val_from), int(val_to),
                                        C.c_void_p(sums.data_ptr()), ow, oh, oll,
                                        C.c_void_p(previews.data_ptr()), oh * oll, _stream_ptr(stream, frames))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_line_preview")
        return previews


def line_batch(frames, width, height, line_length, val_from, val_to, *, band=None, n_frames=None,
               frame_stride=None, stream=None):
    """The ov7670 line sensor over N frames (LSEQ:376-476): sums int64 [N, 3] =
    {points, sum_x, cross points} and targets int8 [N, 4] (targetX, targetY =
    cross size, targetSize).  `band` = the cross-point rows (default: the
    reference's steady state H/2 .. H/2+80)."""
    import torch

    b = _batch(frames, width, height, line_length, LAYOUT_OV7670, n_frames, frame_stride)
    band = (height // 2, height // 2 + 80) if band is None else band
    sums = torch.empty((b.n_frames, 3), dtype=torch.int64, device=frames.device)
    targets = torch.empty((b.n_frames, 4), dtype=torch.int8, device=frames.device)
    rc = _lib.trik_hsv_line_batch(C.byref(b), int(val_from), int(val_to), int(band[0]), int(band[1]),
                                  C.c_void_p(sums.data_ptr()), C.c_void_p(targets.data_ptr()),
                                  _stream_ptr(stream, frames))
    if rc:
        raise TrikHsvError(rc, "trik_hsv_line_batch")
    return sums, targets


def batch_auto_range(frames, width, height, line_length, layout, *, n_frames=None,
                     frame_stride=None, stream=None):
    """autoDetectHsv per frame: uint16 [N, 6] = hue, hueTol, sat, satTol, val, valTol."""
    import torch

    b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
    out = torch.empty((b.n_frames, 6), dtype=torch.int16, device=frames.device)
    rc = _lib.trik_hsv_batch_auto_range(C.byref(b), C.c_void_p(out.data_ptr()), _stream_ptr(stream, frames))
    if rc:
        raise TrikHsvError(rc, "trik_hsv_batch_auto_range")
    return out


def batch_targets(sums, width, height, *, stream=None):
    """Epilogue only: sums int64 [N,T,3] -> targets int8 [N,T,4]."""
    import torch

    N, T = sums.shape[0], sums.shape[1]
    targets = torch.empty((N, T, 4), dtype=torch.int8, device=sums.device)
    b = _abi.FrameBatch(None, 0, N, width, height, 2 * width, LAYOUT_YUYV)
    rc = _lib.trik_hsv_batch_targets(C.byref(b), T, C.c_void_p(sums.data_ptr()),
                                     C.c_void_p(targets.data_ptr()), _stream_ptr(stream, sums))
    if rc:
        raise TrikHsvError(rc, "trik_hsv_batch_targets")
    return targets


def batch_totals_device(sums, *, stream=None):
    """Per-target batch totals on the device (trik_hsv_batch_totals):
    sums int64 [N,T,3] -> [T,3]."""
    import torch

    N, T = sums.shape[0], sums.shape[1]
    totals = torch.empty((T, 3), dtype=torch.int64, device=sums.device)
    rc = _lib.trik_hsv_batch_totals(N, T, C.c_void_p(sums.data_ptr()), C.c_void_p(totals.data_ptr()),
                                    _stream_ptr(stream, sums))
    if rc:
        raise TrikHsvError(rc, "trik_hsv_batch_totals")
    return totals


class Group:
    """One process driving several GPUs through the C ABI's group
    (trik_hsv_group_*): a handle, a stream and a host worker thread per
    device, and one RCCL all-reduce of the per-target totals."""

    def __init__(self, devices):
        self.devices = [int(d) for d in devices]
        arr = (C.c_int32 * len(self.devices))(*self.devices)
        h = C.c_void_p()
        rc = _lib.trik_hsv_group_create(len(self.devices), arr, C.byref(h))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_group_create")
        self._h = h

    def process(self, shards, width, height, line_length, layout, ranges):
        """shards[d]: (frames tensor on devices[d], n_frames).  Returns per
        device (sums [n,T,3], targets [n,T,4], totals [T,3]) -- enqueued on the
        group's streams; call sync() before reading them."""
        import torch

        n = len(self.devices)
        if len(shards) != n:
            raise ValueError("one shard per device")
        arr, T = _ranges(ranges)
        batches = (_abi.FrameBatch * n)()
        out, keep = [], []
        for d, (frames, nf) in enumerate(shards):
            dev = torch.device("cuda", self.devices[d])
            batches[d] = _batch(frames, width, height, line_length, layout, nf)
            sums = torch.zeros((max(nf, 0), T, 3), dtype=torch.int64, device=dev)
            targets = torch.zeros((max(nf, 0), T, 4), dtype=torch.int8, device=dev)
            totals = torch.zeros((T, 3), dtype=torch.int64, device=dev)
            out.append((sums, targets, totals))
        torch.cuda.synchronize()  # the allocations above ran on torch's streams
        ptrs = [(C.c_void_p * n)(*[C.c_void_p(o[k].data_ptr()) for o in out]) for k in range(3)]
        rc = _lib.trik_hsv_group_process(self._h, batches, arr, T, ptrs[0], ptrs[1], ptrs[2])
        if rc:
            raise TrikHsvError(rc, "trik_hsv_group_process")
        self._keep = (batches, ptrs, out)
        return out

    def sync(self):
        rc = _lib.trik_hsv_group_sync(self._h)
        if rc:
            raise TrikHsvError(rc, "trik_hsv_group_sync")

    def close(self):
        if getattr(self, "_h", None):
            _lib.trik_hsv_group_delete(self._h)
            self._h = None

    def __del__(self):
        self.close()


COMM_ID_BYTES = 128  # TRIK_HSV_COMM_ID_BYTES (= NCCL_UNIQUE_ID_BYTES)


def comm_id() -> bytes:
    """A fresh communicator id (rank 0 makes it; every rank passes the same
    bytes to Comm): trik_hsv_comm_id."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    rc = _lib.trik_hsv_comm_id(buf)
    if rc:
        raise TrikHsvError(rc, "trik_hsv_comm_id")
    return bytes(buf)


class Comm:
    """One process per GPU: the library's own RCCL communicator over the ranks
    (trik_hsv_comm_create on the current device) and its one collective, the
    sum of the per-target totals (trik_hsv_comm_all_reduce_totals) -- the call
    a C++ host links, not torch.distributed's."""

    def __init__(self, n_ranks: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"comm id must be {COMM_ID_BYTES} bytes")
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        rc = _lib.trik_hsv_comm_create(int(n_ranks), int(rank), buf, C.byref(h))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_comm_create")
        self._h = h
        self.n_ranks, self.rank = int(n_ranks), int(rank)

    def all_reduce_totals(self, totals, *, stream=None):
        """Sum totals [T, 3] int64 (device) over the ranks in place, enqueued
        on `stream` (default: torch's current stream)."""
        import torch

        if totals.dtype != torch.int64 or totals.dim() != 2 or totals.shape[1] != 3 or not totals.is_contiguous():
            raise ValueError("totals must be a contiguous [T, 3] int64 device tensor")
        rc = _lib.trik_hsv_comm_all_reduce_totals(self._h, C.c_void_p(totals.data_ptr()), int(totals.shape[0]),
                                                  _stream_ptr(stream, totals))
        if rc:
            raise TrikHsvError(rc, "trik_hsv_comm_all_reduce_totals")
        return totals

    def close(self):
        if getattr(self, "_h", None):
            _lib.trik_hsv_comm_delete(self._h)
            self._h = None

    def __del__(self):
        self.close()


def synth(frames, width, height, line_length, layout, kind, seed, *, first_frame=0, n_frames=None,
          frame_stride=None, stream=None):
    """Fill a uint8 device tensor with synthetic frames (kind 0 uniform, 1 scene)."""
    b = _batch(frames, width, height, line_length, layout, n_frames, frame_stride)
    rc = _lib.trik_hsv_synth(C.byref(b), first_frame, kind, seed, _stream_ptr(stream, frames))
    if rc:
        raise TrikHsvError(rc, "trik_hsv_synth")
    return frames


# ---------------------------------------------------------------------------
# ObjectSensor: the codec instance (XDAIS quartet)
# ---------------------------------------------------------------------------
def _default_params(num_output_streams=1, fmt_in=FORMAT_YUV422, max_w=640, max_h=480):
    """TRIK_VIDTRANSCODE_CV_Params defaults (WGLUE:153-184), caps adjustable."""
    p = _abi.Params()
    b = p.base
    b.size = C.sizeof(_abi.Params)
    b.numOutputStreams = num_output_streams
    b.formatInput = fmt_in
    b.formatOutput[0], b.formatOutput[1] = (FORMAT_RGB565X if num_output_streams else FORMAT_UNKNOWN,
                                            FORMAT_UNKNOWN)
    b.maxHeightInput, b.maxWidthInput, b.maxFrameRateInput, b.maxBitRateInput = max_h, max_w, 60000, -1
    b.maxHeightOutput[0], b.maxHeightOutput[1] = max_h, -1
    b.maxWidthOutput[0], b.maxWidthOutput[1] = max_w, -1
    b.maxFrameRateOutput[0] = b.maxFrameRateOutput[1] = -1
    b.maxBitRateOutput[0] = b.maxBitRateOutput[1] = -1
    b.dataEndianness = 1
    if num_output_streams == 0:  # caps checks still read index 0
        b.maxHeightOutput[0], b.maxWidthOutput[0] = max_h, max_w
    return p


def dynamic_params(width, height, line_length, out_width=320, out_height=240, out_line_length=640):
    d = _abi.DynamicParams()
    d.base.size = C.sizeof(_abi.DynamicParams)
    d.base.keepInputResolutionFlag[1] = 1
    d.base.outputHeight[0], d.base.outputWidth[0] = out_height, out_width
    d.base.keepInputFrameRateFlag[0] = d.base.keepInputFrameRateFlag[1] = 1
    d.base.inputFrameRate = -1
    d.base.forceFrame[0] = d.base.forceFrame[1] = -1
    d.inputHeight, d.inputWidth, d.inputLineLength = height, width, line_length
    d.outputLineLength[0], d.outputLineLength[1] = out_line_length, -1
    return d


class ObjectSensor(_HotKernel):
    """One TRIK_VIDTRANSCODE_CV codec instance (vidtranscode_cv_fxns.c)."""

    _create = "TRIK_VIDTRANSCODE_CV_create"

    def __init__(self, params: _abi.Params | None = None):
        h = C.c_void_p()
        rc = getattr(_lib, self._create)(C.byref(params) if params is not None else None, C.byref(h))
        if rc != IALG_EOK:
            raise TrikHsvError(rc, self._create)
        self._h = h
        self.params = params if params is not None else _default_params(1)

    def close(self):
        if getattr(self, "_h", None):
            _lib.TRIK_VIDTRANSCODE_CV_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def control(self, cmd: int, dyn: _abi.DynamicParams | None = None,
                status: _abi.Status | None = None):
        st = status if status is not None else _abi.Status()
        rc = _lib.TRIK_VIDTRANSCODE_CV_control(self._h, cmd, C.byref(dyn) if dyn is not None else None,
                                               C.byref(st))
        return rc, st

    def set_params(self, width, height, line_length, **kw) -> int:
        rc, _ = self.control(XDM_SETPARAMS, dynamic_params(width, height, line_length, **kw))
        return rc

    def process(self, frame, hsv_range: Sequence[int], out_buffer=None, auto_detect=False,
                num_bytes=None, input_id=0):
        """One host frame (bytes / numpy uint8) -> (rc, OutArgs)."""
        import numpy as np

        fr = np.ascontiguousarray(np.frombuffer(frame, np.uint8) if isinstance(frame, (bytes, bytearray))
                                  else frame, dtype=np.uint8)
        ib = _abi.BufDesc1()
        ib.numBufs = 1
        ib.descs[0].buf = fr.ctypes.data
        ib.descs[0].bufSize = fr.size
        ob = _abi.BufDesc()
        keep = []
        if out_buffer is not None:
            ob_arr = (C.c_void_p * 1)(out_buffer.ctypes.data)
            sz_arr = (C.c_int32 * 1)(out_buffer.nbytes)
            keep += [ob_arr, sz_arr]
            ob.bufs, ob.numBufs, ob.bufSizes = ob_arr, 1, sz_arr
        ia = _abi.InArgs()
        ia.base.size = C.sizeof(_abi.InArgs)
        ia.base.numBytes = fr.size if num_bytes is None else num_bytes
        ia.base.inputID = input_id
        ia.alg = _abi.InArgsAlg(*[int(v) for v in hsv_range[:6]], int(bool(auto_detect)))
        oa = _abi.OutArgs()
        oa.base.size = C.sizeof(_abi.OutArgs)
        rc = _lib.TRIK_VIDTRANSCODE_CV_process(self._h, C.byref(ib), C.byref(ob), C.byref(ia),
                                               C.byref(oa))
        return rc, oa

    def _bufs(self, frame, out_buffer, num_bytes):
        import numpy as np

        fr = np.ascontiguousarray(np.frombuffer(frame, np.uint8) if isinstance(frame, (bytes, bytearray))
                                  else frame, dtype=np.uint8)
        ib = _abi.BufDesc1()
        ib.numBufs = 1
        ib.descs[0].buf = fr.ctypes.data
        ib.descs[0].bufSize = fr.size
        ob = _abi.BufDesc()
        keep = [fr]
        if out_buffer is not None:
            ob_arr = (C.c_void_p * 1)(out_buffer.ctypes.data)
            sz_arr = (C.c_int32 * 1)(out_buffer.nbytes)
            keep += [ob_arr, sz_arr]
            ob.bufs, ob.numBufs, ob.bufSizes = ob_arr, 1, sz_arr
        return fr, ib, ob, keep


class LineSensor(ObjectSensor):
    """The ov7670 line sensor's codec instance (trik/ov7670/line_sensor glue,
    LineDetector<YUV422P, RGB565X>): same quartet, YUV422P input; process()
    uses only detectValFrom/To of the range and ignores autoDetectHsv; OutArgs
    targetY carries the cross size."""

    _create = "TRIK_VIDTRANSCODE_CV_create_line"

    def __init__(self, params: _abi.Params | None = None):
        super().__init__(params)
        if params is None:
            self.params = _default_params(1, fmt_in=FORMAT_YUV422P)


class WebcamLineSensor(ObjectSensor):
    """The webcam line sensor's codec instance (trik/webcam/line_sensor glue,
    LineDetector<YUV422, RGB565X>): same quartet and InArgs/OutArgs as the
    object sensor, packed YUYV input; process() uses only detectValFrom/To,
    targetY is always 0, autoDetectHsv is ignored."""

    _create = "TRIK_VIDTRANSCODE_CV_create_webcam_line"


class BlobSensor(ObjectSensor):
    """The ov7670 object sensor's codec instance (trik/ov7670/object_sensor:
    BallDetector<YUV422P, RGB565X> with BitmapBuilder + Clusterizer): its own
    InArgs (centre/tolerance, sticky via setHsvRange) and OutArgs (target[8])."""

    _create = "TRIK_VIDTRANSCODE_CV_create_ov7670"

    def __init__(self, params: _abi.Params | None = None):
        super().__init__(params)
        if params is None:
            self.params = _default_params(1, fmt_in=FORMAT_YUV422P)

    def process(self, frame, hsv=None, out_buffer=None, auto_detect=False, num_bytes=None, input_id=0):
        """One host frame -> (rc, OV7670OutArgs).  hsv = (hue, hueTol, sat,
        satTol, val, valTol) sets the range (setHsvRange); None keeps it."""
        fr, ib, ob, keep = self._bufs(frame, out_buffer, num_bytes)
        ia = _abi.OV7670InArgs()
        ia.base.size = C.sizeof(_abi.OV7670InArgs)
        ia.base.numBytes = fr.size if num_bytes is None else num_bytes
        ia.base.inputID = input_id
        vals = [int(v) for v in hsv] if hsv is not None else [0] * 6
        ia.alg = _abi.OV7670InArgsAlg(1 if hsv is not None else 0, *vals, int(bool(auto_detect)))
        oa = _abi.OV7670OutArgs()
        oa.base.size = C.sizeof(_abi.OV7670OutArgs)
        rc = _lib.TRIK_VIDTRANSCODE_CV_process(self._h, C.byref(ib), C.byref(ob), C.byref(ia), C.byref(oa))
        return rc, oa
