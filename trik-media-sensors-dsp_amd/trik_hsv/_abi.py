"""ctypes mirror of include/trik_hsv.h (the C ABI of libtrik_hsv.so).

The library is the product: HIP kernels for gfx950 plus the C++ XDAIS-shaped
host layer.  This module only declares its structs and entry points; there is
no fallback -- if the library is missing, importing trik_hsv fails.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtrik_hsv.so")
CSRC = os.path.join(os.path.dirname(HERE), "csrc")

# return codes / commands / bits (TI ialg.h, xdm.h values)
IALG_EOK = 0
IALG_EFAIL = -1
IVIDTRANSCODE_EOK = 0
IVIDTRANSCODE_EFAIL = -1
IVIDTRANSCODE_EUNSUPPORTED = -3
XDM_GETSTATUS, XDM_SETPARAMS, XDM_RESET, XDM_SETDEFAULT, XDM_FLUSH, XDM_GETBUFINFO, XDM_GETVERSION = range(7)
XDM_CORRUPTEDDATA_BIT = 11
XDM_UNSUPPORTEDPARAM_BIT = 14
XDM_ACCESSMODE_READ = 0
XDM_ACCESSMODE_WRITE = 1
XDM_CUSTOMENUMBASE = 0x100
FORMAT_UNKNOWN = 0
FORMAT_RGB888 = XDM_CUSTOMENUMBASE
FORMAT_RGB565 = XDM_CUSTOMENUMBASE + 1
FORMAT_RGB565X = XDM_CUSTOMENUMBASE + 2
FORMAT_YUV444 = XDM_CUSTOMENUMBASE + 3
FORMAT_YUV422 = XDM_CUSTOMENUMBASE + 4
FORMAT_YUV422P = XDM_CUSTOMENUMBASE + 5
MAXOUTSTREAMS = 2
MAX_IO_BUFFERS = 16
LAYOUT_YUYV = 0
LAYOUT_OV7670 = 1
MAX_RANGES = 64

i32, i64, u8, u16, u64 = C.c_int32, C.c_int64, C.c_uint8, C.c_uint16, C.c_uint64
A2 = i32 * MAXOUTSTREAMS


class IVidtranscodeParams(C.Structure):
    _fields_ = [("size", i32), ("numOutputStreams", i32), ("formatInput", i32),
                ("formatOutput", A2), ("maxHeightInput", i32), ("maxWidthInput", i32),
                ("maxFrameRateInput", i32), ("maxBitRateInput", i32), ("maxHeightOutput", A2),
                ("maxWidthOutput", A2), ("maxFrameRateOutput", A2), ("maxBitRateOutput", A2),
                ("dataEndianness", i32)]


class Params(C.Structure):
    _fields_ = [("base", IVidtranscodeParams)]


class IVidtranscodeDynamicParams(C.Structure):
    _fields_ = [("size", i32), ("readHeaderOnlyFlag", i32), ("keepInputResolutionFlag", A2),
                ("outputHeight", A2), ("outputWidth", A2), ("keepInputFrameRateFlag", A2),
                ("inputFrameRate", i32), ("outputFrameRate", A2), ("targetBitRate", A2),
                ("rateControl", A2), ("keepInputGOPFlag", A2), ("intraFrameInterval", A2),
                ("interFrameInterval", A2), ("forceFrame", A2), ("frameSkipTranscodeFlag", A2)]


class DynamicParams(C.Structure):
    _fields_ = [("base", IVidtranscodeDynamicParams), ("inputHeight", i32), ("inputWidth", i32),
                ("inputLineLength", i32), ("outputLineLength", A2)]


class InArgsAlg(C.Structure):
    """TRIK_VIDTRANSCODE_CV_InArgsAlg (webcam trik_vidtranscode_cv.h:48-56)."""
    _fields_ = [("detectHueFrom", u16), ("detectHueTo", u16), ("detectSatFrom", u8),
                ("detectSatTo", u8), ("detectValFrom", u8), ("detectValTo", u8),
                ("autoDetectHsv", i32)]


class IVidtranscodeInArgs(C.Structure):
    _fields_ = [("size", i32), ("numBytes", i32), ("inputID", i32)]


class InArgs(C.Structure):
    _fields_ = [("base", IVidtranscodeInArgs), ("alg", InArgsAlg)]



class OutArgsAlg(C.Structure):
    """TRIK_VIDTRANSCODE_CV_OutArgsAlg (webcam trik_vidtranscode_cv.h:64-74)."""
    _fields_ = [("targetX", C.c_int8), ("targetY", C.c_int8), ("targetSize", u8),
                ("detectHue", u16), ("detectHueTolerance", u16), ("detectSat", u16),
                ("detectSatTolerance", u16), ("detectVal", u16), ("detectValTolerance", u16)]


class OV7670InArgsAlg(C.Structure):
    """TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg (ov7670 object sensor trik_vidtranscode_cv.h:51-60)."""
    _fields_ = [("setHsvRange", i32), ("detectHue", u16), ("detectHueTol", u16), ("detectSat", u8),
                ("detectSatTol", u8), ("detectVal", u8), ("detectValTol", u8), ("autoDetectHsv", i32)]


class XdasTarget(C.Structure):
    _fields_ = [("x", C.c_int8), ("y", C.c_int8), ("size", u8)]


class OV7670OutArgsAlg(C.Structure):
    """TRIK_VIDTRANSCODE_CV_OV7670_OutArgsAlg (ov7670 trik_vidtranscode_cv.h:73-81)."""
    _fields_ = [("target", XdasTarget * 8), ("detectHue", u16), ("detectHueTolerance", u16),
                ("detectSat", u16), ("detectSatTolerance", u16), ("detectVal", u16),
                ("detectValTolerance", u16)]


class SingleBufDesc(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("bufSize", i32), ("accessMask", i32)]


class BufDesc1(C.Structure):
    _fields_ = [("numBufs", i32), ("descs", SingleBufDesc * MAX_IO_BUFFERS)]


class BufDesc(C.Structure):
    _fields_ = [("bufs", C.POINTER(C.c_void_p)), ("numBufs", i32), ("bufSizes", C.POINTER(i32))]


class IVidtranscodeOutArgs(C.Structure):
    _fields_ = [("size", i32), ("extendedError", i32), ("bitsConsumed", i32),
                ("decodedPictureType", i32), ("decodedPictureStructure", i32),
                ("decodedHeight", i32), ("decodedWidth", i32),
                ("encodedBuf", SingleBufDesc * MAXOUTSTREAMS), ("bitsGenerated", A2),
                ("encodedPictureType", A2), ("encodedPictureStructure", A2), ("outputID", A2),
                ("inputFrameSkipTranscodeFlag", A2), ("outBufsInUseFlag", i32)]


class OutArgs(C.Structure):
    _fields_ = [("base", IVidtranscodeOutArgs), ("alg", OutArgsAlg)]


class OV7670InArgs(C.Structure):
    _fields_ = [("base", IVidtranscodeInArgs), ("alg", OV7670InArgsAlg)]


class OV7670OutArgs(C.Structure):
    _fields_ = [("base", IVidtranscodeOutArgs), ("alg", OV7670OutArgsAlg)]


class AlgBufInfo(C.Structure):
    _fields_ = [("minNumInBufs", i32), ("minNumOutBufs", i32),
                ("minInBufSize", i32 * MAX_IO_BUFFERS), ("minOutBufSize", i32 * MAX_IO_BUFFERS)]


class Status(C.Structure):
    _fields_ = [("size", i32), ("extendedError", i32), ("data", SingleBufDesc),
                ("bufInfo", AlgBufInfo)]


class FrameBatch(C.Structure):
    _fields_ = [("frames", C.c_void_p), ("frame_stride", i64), ("n_frames", i32),
                ("width", i32), ("height", i32), ("line_length", i32), ("layout", i32)]


class TargetSums(C.Structure):
    _fields_ = [("points", i64), ("sum_x", i64), ("sum_y", i64)]


class Target(C.Structure):
    _fields_ = [("x", C.c_int8), ("y", C.c_int8), ("size", u8), ("reserved", u8)]


# every symbol include/trik_hsv.h declares, with its prototype
PROTOTYPES = {
    "TRIK_VIDTRANSCODE_CV_create": ([C.POINTER(Params), C.POINTER(C.c_void_p)], i32),
    "TRIK_VIDTRANSCODE_CV_create_line": ([C.POINTER(Params), C.POINTER(C.c_void_p)], i32),
    "TRIK_VIDTRANSCODE_CV_create_ov7670": ([C.POINTER(Params), C.POINTER(C.c_void_p)], i32),
    "TRIK_VIDTRANSCODE_CV_create_webcam_line": ([C.POINTER(Params), C.POINTER(C.c_void_p)], i32),
    "TRIK_VIDTRANSCODE_CV_delete": ([C.c_void_p], i32),
    # InArgs / OutArgs by pointer: the webcam structs, or the OV7670 ones for
    # a create_ov7670 handle (their base.size fields say which)
    "TRIK_VIDTRANSCODE_CV_process": ([C.c_void_p, C.POINTER(BufDesc1), C.POINTER(BufDesc),
                                      C.c_void_p, C.c_void_p], i32),
    "TRIK_VIDTRANSCODE_CV_control": ([C.c_void_p, i32, C.POINTER(DynamicParams),
                                      C.POINTER(Status)], i32),
    "trik_hsv_version": ([], C.c_char_p),
    "trik_hsv_last_error": ([], C.c_char_p),
    "trik_hsv_process_batch": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(InArgsAlg), i32,
                                C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "trik_hsv_process_batch_totals": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(InArgsAlg), i32,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "trik_hsv_batch_sums": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(InArgsAlg), i32,
                             C.c_void_p, C.c_void_p], i32),
    "trik_hsv_batch_targets": ([C.POINTER(FrameBatch), i32, C.c_void_p, C.c_void_p,
                                C.c_void_p], i32),
    "trik_hsv_batch_masks": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(InArgsAlg), i32,
                              C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "trik_hsv_batch_preview": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(InArgsAlg), C.c_void_p,
                                i32, i32, i32, i32, C.c_void_p, C.c_int64, C.c_void_p], i32),
    "trik_hsv_batch_auto_range": ([C.POINTER(FrameBatch), C.c_void_p, C.c_void_p], i32),
    "trik_hsv_line_batch": ([C.POINTER(FrameBatch), i32, i32, i32, i32, C.c_void_p, C.c_void_p,
                             C.c_void_p], i32),
    "trik_hsv_line_preview": ([C.c_void_p, C.POINTER(FrameBatch), i32, i32, C.c_void_p, i32, i32, i32,
                               C.c_void_p, C.c_int64, C.c_void_p], i32),
    "trik_hsv_blob_batch": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(OV7670InArgsAlg), C.c_void_p,
                             C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "trik_hsv_blob_preview": ([C.c_void_p, C.POINTER(FrameBatch), C.c_void_p, C.c_void_p, i32, i32, i32,
                               C.c_void_p, C.c_int64, C.c_void_p], i32),
    "trik_hsv_synth": ([C.POINTER(FrameBatch), i32, i32, u64, C.c_void_p], i32),
    "trik_hsv_set_hot_kernel": ([C.c_void_p, i32], i32),
    "trik_hsv_last_hot_kernel": ([C.c_void_p], i32),
    "trik_hsv_set_reserved_cus": ([C.c_void_p, i32], i32),
    "trik_hsv_chroma_share": ([C.c_void_p, C.POINTER(C.c_double)], i32),
    "trik_hsv_chroma_measured_share": ([C.c_void_p, C.POINTER(C.c_double)], i32),
    # XDAIS IALG functions (also in the exported function tables)
    "TRIK_VIDTRANSCODE_CV_alloc": ([C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "TRIK_VIDTRANSCODE_CV_initObj": ([C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "TRIK_VIDTRANSCODE_CV_free": ([C.c_void_p, C.c_void_p], i32),
    # multi-GPU layer
    "trik_hsv_batch_totals": ([i32, i32, C.c_void_p, C.c_void_p, C.c_void_p], i32),
    "trik_hsv_group_create": ([i32, C.POINTER(i32), C.POINTER(C.c_void_p)], i32),
    "trik_hsv_group_process": ([C.c_void_p, C.POINTER(FrameBatch), C.POINTER(InArgsAlg), i32,
                                C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)], i32),
    "trik_hsv_group_sync": ([C.c_void_p], i32),
    "trik_hsv_group_stream": ([C.c_void_p, i32], C.c_void_p),
    "trik_hsv_group_delete": ([C.c_void_p], i32),
    "trik_hsv_comm_id": ([C.c_void_p], i32),
    "trik_hsv_comm_create": ([i32, i32, C.c_void_p, C.POINTER(C.c_void_p)], i32),
    "trik_hsv_comm_all_reduce_totals": ([C.c_void_p, C.c_void_p, i32, C.c_void_p], i32),
    "trik_hsv_comm_delete": ([C.c_void_p], i32),
}

_lib = None


def load() -> C.CDLL:
    """Load libtrik_hsv.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 /
        # libhsa-runtime64 (same SONAME, loaded by path).  If this library loaded
        # /opt/rocm's first, importing torch afterwards would map a second HSA
        # runtime and this library's would see no device.  Loading torch first
        # makes the library's DT_NEEDED libamdhip64.so.7 bind to torch's copy.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C {CSRC}` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in PROTOTYPES.items():
            fn = getattr(L, name)
            fn.argtypes, fn.restype = args, res
        _lib = L
    return _lib


def last_error() -> str:
    return load().trik_hsv_last_error().decode(errors="replace")
