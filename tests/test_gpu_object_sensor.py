"""The XDAIS-shaped codec surface (create / control / process / delete) on the
GPU: same OutArgs as the oracle, same return codes and extendedError bits as
trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c."""
import ctypes as C

import numpy as np
import pytest

from gpu_util import LAYOUT_OV7670, LAYOUT_YUYV, T0, T3

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hsv():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import trik_hsv

    return trik_hsv


def test_default_instance_and_version(hsv):
    s = hsv.ObjectSensor()
    st = hsv._abi.Status()
    buf = C.create_string_buffer(32)
    st.data.buf = C.cast(buf, C.c_void_p)
    st.data.bufSize = 32
    rc, st = s.control(hsv.XDM_GETVERSION, status=st)
    assert rc == 0 and buf.value == b"1.00.00.00"
    st.data.bufSize = 4
    rc, _ = s.control(hsv.XDM_GETVERSION, status=st)
    assert rc == hsv.IVIDTRANSCODE_EFAIL
    rc, st = s.control(hsv.XDM_GETBUFINFO)
    assert rc == 0 and st.bufInfo.minNumInBufs == 1 and st.bufInfo.minNumOutBufs == 1
    assert rc == 0 and s.control(hsv.XDM_FLUSH)[0] == 0
    assert s.control(99)[0] == hsv.IVIDTRANSCODE_EFAIL
    s.close()


@pytest.mark.parametrize("kind,rng", [(0, T0), (1, T0), (1, T3)])
def test_process_matches_oracle(hsv, oracle_mod, kind, rng):
    w, h, ll = 640, 480, 1280
    s = hsv.ObjectSensor()
    assert s.set_params(w, h, ll) == 0
    frame = oracle_mod.synth(1, w, h, ll, LAYOUT_YUYV, kind, 0x7A1C, first_frame=9)
    out = np.full(240 * 640 + 64, 0xAB, np.uint8)
    rc, oa = s.process(frame, rng, out_buffer=out)
    assert rc == 0
    want = oracle_mod.targets(oracle_mod.frame(frame, w, h, ll, LAYOUT_YUYV, [rng])[0][0], w, h)
    assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == want
    assert oa.base.encodedBuf[0].bufSize == 240 * 640          # WSEQ:419
    assert oa.base.bitsConsumed == frame.size * 8
    assert oa.base.outputID[0] == 0 and oa.base.outBufsInUseFlag == 0
    _, _, preview = oracle_mod.run(frame, w, h, ll, LAYOUT_YUYV, rng)
    assert np.array_equal(out[:240 * 640], preview)            # rendered preview (WSEQ:316-354)
    assert not out[240 * 640:].any()                            # rest zero-filled (WFXNS:234)
    s.close()


def test_ov7670_instance(hsv, oracle_mod):
    p = hsv._default_params(1, fmt_in=hsv.FORMAT_YUV422P, max_w=320, max_h=240)
    s = hsv.ObjectSensor(p)
    assert s.set_params(320, 240, 320) == 0
    frame = oracle_mod.synth(1, 320, 240, 320, LAYOUT_OV7670, 1, 5)
    rc, oa = s.process(frame, T0, out_buffer=np.zeros(240 * 640, np.uint8))
    assert rc == 0
    want = oracle_mod.targets(oracle_mod.frame(frame, 320, 240, 320, LAYOUT_OV7670, [T0])[0][0], 320, 240)
    assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == want


def test_error_codes(hsv):
    s = hsv.ObjectSensor()
    assert s.set_params(640, 480, 1280) == 0
    frame = np.zeros(640 * 480 * 2, np.uint8)
    out = np.zeros(240 * 640, np.uint8)
    # input smaller than H*lineLength -> EFAIL + XDM_CORRUPTEDDATA (WSEQ:415, WFXNS:243-247)
    rc, oa = s.process(frame[:1000], T0, out_buffer=out)
    assert rc == hsv.IVIDTRANSCODE_EFAIL
    assert oa.base.extendedError & (1 << hsv._abi.XDM_CORRUPTEDDATA_BIT)
    # numBytes > bufSize -> EFAIL + XDM_UNSUPPORTEDPARAM (WFXNS:207-214)
    rc, oa = s.process(frame, T0, out_buffer=out, num_bytes=frame.size + 1)
    assert rc == hsv.IVIDTRANSCODE_EFAIL
    assert oa.base.extendedError & (1 << hsv._abi.XDM_UNSUPPORTEDPARAM_BIT)
    # SETPARAMS with wrong struct size -> EUNSUPPORTED (WFXNS:300-305)
    d = hsv.dynamic_params(640, 480, 1280)
    d.base.size = 12
    assert s.control(hsv.XDM_SETPARAMS, d)[0] == hsv.IVIDTRANSCODE_EUNSUPPORTED
    # geometry the reference's setup rejects (W % 32) -> EFAIL, then process fails too
    assert s.set_params(630, 480, 1260) == hsv.IALG_EFAIL
    rc, _ = s.process(frame, T0, out_buffer=out)
    assert rc == hsv.IVIDTRANSCODE_EFAIL
    # over the max dimensions of the instance
    assert s.set_params(1280, 720, 2560) == hsv.IALG_EFAIL
    # RESET restores the default (0x0 input): process succeeds with zero targets
    assert s.control(hsv.XDM_RESET)[0] == 0
    rc, oa = s.process(frame, T0, out_buffer=out)
    assert rc == 0 and (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == (0, 0, 0)
    s.close()


def test_zero_output_streams(hsv, oracle_mod):
    p = hsv._default_params(0)
    s = hsv.ObjectSensor(p)
    assert s.set_params(640, 480, 1280) == 0
    frame = oracle_mod.synth(1, 640, 480, 1280, LAYOUT_YUYV, 1, 3)
    rc, oa = s.process(frame, T0)
    assert rc == 0
    want = oracle_mod.targets(oracle_mod.frame(frame, 640, 480, 1280, LAYOUT_YUYV, [T0])[0][0], 640, 480)
    assert (oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize) == want
