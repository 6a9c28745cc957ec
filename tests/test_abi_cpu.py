"""CPU-only checks of the C ABI: the library loads, exports every function
include/trik_hsv.h declares, and the ctypes mirror has the C layout.  No
compute calls (there is no GPU here)."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "trik_hsv.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(\w+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "while")))


@pytest.fixture(scope="module")
def abi():
    from trik_hsv import _abi

    return _abi


def test_header_declares_the_quartet_and_batch_api():
    names = declared_functions()
    for n in ("TRIK_VIDTRANSCODE_CV_create", "TRIK_VIDTRANSCODE_CV_delete",
              "TRIK_VIDTRANSCODE_CV_process", "TRIK_VIDTRANSCODE_CV_control",
              "trik_hsv_process_batch", "trik_hsv_batch_sums", "trik_hsv_batch_targets",
              "trik_hsv_batch_masks", "trik_hsv_synth", "trik_hsv_version", "trik_hsv_last_error",
              "TRIK_VIDTRANSCODE_CV_create_line", "TRIK_VIDTRANSCODE_CV_create_ov7670",
              "TRIK_VIDTRANSCODE_CV_create_webcam_line",
              "trik_hsv_line_batch", "trik_hsv_line_preview", "trik_hsv_blob_batch", "trik_hsv_blob_preview",
              "trik_hsv_batch_preview", "trik_hsv_batch_auto_range"):
        assert n in names


def test_library_exports_every_declared_symbol(abi):
    lib = abi.load()
    for n in declared_functions():
        assert hasattr(lib, n), n
        assert n in abi.PROTOTYPES, f"ctypes mirror lacks {n}"


def test_version_without_gpu(abi):
    assert b"gfx950" in abi.load().trik_hsv_version()
    assert abi.load().trik_hsv_last_error() == b""


def test_set_reserved_cus_rejects_without_gpu(abi):
    """trik_hsv_set_reserved_cus validates before touching a handle: a NULL
    handle or a count outside 0..32 returns -1 (no GPU needed)."""
    lib = abi.load()
    for n in (0, 2, 32, -1, 33):
        assert lib.trik_hsv_set_reserved_cus(None, n) == -1


STRUCTS = ["TRIK_VIDTRANSCODE_CV_Params", "TRIK_VIDTRANSCODE_CV_DynamicParams",
           "TRIK_VIDTRANSCODE_CV_InArgsAlg", "TRIK_VIDTRANSCODE_CV_InArgs",
           "TRIK_VIDTRANSCODE_CV_OutArgsAlg", "TRIK_VIDTRANSCODE_CV_OutArgs",
           "TRIK_XDM1_BufDesc", "TRIK_XDM_BufDesc", "TRIK_IVIDTRANSCODE_Status",
           "TrikHsvFrameBatch", "TrikHsvTargetSums", "TrikHsvTarget",
           "TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg", "TRIK_VIDTRANSCODE_CV_OV7670_InArgs",
           "TRIK_XDAS_Target", "TRIK_VIDTRANSCODE_CV_OV7670_OutArgsAlg", "TRIK_VIDTRANSCODE_CV_OV7670_OutArgs"]
MIRRORS = ["Params", "DynamicParams", "InArgsAlg", "InArgs", "OutArgsAlg", "OutArgs",
           "BufDesc1", "BufDesc", "Status", "FrameBatch", "TargetSums", "Target",
           "OV7670InArgsAlg", "OV7670InArgs", "XdasTarget", "OV7670OutArgsAlg", "OV7670OutArgs"]


def test_struct_layout_matches_c(abi):
    prog = "#include <stdio.h>\n#include \"trik_hsv.h\"\nint main(void){\n"
    for s in STRUCTS:
        prog += f'  printf("%zu\\n", sizeof({s}));\n'
    prog += '  printf("%zu %zu %zu %zu\\n", offsetof(TRIK_VIDTRANSCODE_CV_OV7670_OutArgs, alg), ' \
            'offsetof(TRIK_VIDTRANSCODE_CV_OV7670_InArgs, alg), ' \
            'offsetof(TRIK_VIDTRANSCODE_CV_OutArgs, alg), offsetof(TRIK_VIDTRANSCODE_CV_InArgs, alg));\n' \
            '  return 0;\n}\n'
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "sz.c")
        open(c, "w").write(prog.replace("#include <stdio.h>", "#include <stdio.h>\n#include <stddef.h>"))
        exe = os.path.join(d, "sz")
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    sizes = [int(x) for x in out[: len(STRUCTS)]]
    for s, m, n in zip(STRUCTS, MIRRORS, sizes):
        assert C.sizeof(getattr(abi, m)) == n, (s, C.sizeof(getattr(abi, m)), n)
    assert int(out[-2]) == abi.OutArgs.alg.offset and int(out[-1]) == abi.InArgs.alg.offset
    assert int(out[-4]) == abi.OV7670OutArgs.alg.offset and int(out[-3]) == abi.OV7670InArgs.alg.offset


def test_header_compiles_as_cxx():
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "h.cpp")
        open(c, "w").write('#include "trik_hsv.h"\nint main(){return TRIK_IALG_EOK;}\n')
        subprocess.run(["g++", "-std=c++11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        c, "-o", os.path.join(d, "h")], check=True)


XDAIS_PROG = r"""
#include <stdio.h>
#include <stdlib.h>
#include "trik_hsv.h"
/* a Codec-Engine-style caller that binds only the function tables */
int main(void) {
  const TRIK_IVIDTRANSCODE_Fxns* tabs[4] = {&TRIK_VIDTRANSCODE_CV_FXNS, &TRIK_VIDTRANSCODE_CV_OV7670_FXNS,
                                            &TRIK_VIDTRANSCODE_CV_LINE_FXNS, &TRIK_VIDTRANSCODE_CV_WEBCAM_LINE_FXNS};
  for (int i = 0; i < 4; ++i) {
    const TRIK_IVIDTRANSCODE_Fxns* f = tabs[i];
    TRIK_IALG_MemRec m[16];
    TRIK_IALG_Fxns* parent = NULL;
    int n = f->ialg.algAlloc(NULL, &parent, m);
    if (n != 1 || m[0].size < sizeof(TRIK_IALG_Obj) || m[0].attrs != TRIK_IALG_PERSIST) return 10 + i;
    if (f->ialg.implementationId != (const void*)f || !f->process || !f->control || !f->ialg.algInit ||
        !f->ialg.algFree || f->ialg.algActivate || f->ialg.algNumAlloc) return 20 + i;
    printf("%d %u %d\n", n, m[0].size, m[0].alignment);
  }
  if (TRIK_VIDTRANSCODE_CV_IALG.algAlloc != TRIK_VIDTRANSCODE_CV_FXNS.ialg.algAlloc ||
      TRIK_VIDTRANSCODE_CV_IALG.implementationId != (const void*)&TRIK_VIDTRANSCODE_CV_FXNS) return 30;
  return 0;
}
"""


def test_xdais_tables_link_from_c_and_alloc_without_gpu():
    """The exported XDAIS tables (WFXNS:20-66) bind from plain C; algAlloc
    needs no device."""
    lib_dir = os.path.join(ROOT, "trik-media-sensors-dsp_amd", "trik_hsv")
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "x.c"), os.path.join(d, "x")
        open(c, "w").write(XDAIS_PROG)
        subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{os.path.join(ROOT, 'include')}", c,
                        f"-L{lib_dir}", "-ltrik_hsv", f"-Wl,-rpath,{lib_dir}", "-o", exe], check=True)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert len(r.stdout.split("\n")) >= 4


XDAIS_FAIL_PROG = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "trik_hsv.h"
/* TI's ALG_create after a failed algInit: algFree on the same record, which
 * must find a valid object (destroyed once), then the record is released. */
int main(void) {
  const TRIK_IVIDTRANSCODE_Fxns* f = &TRIK_VIDTRANSCODE_CV_FXNS;
  TRIK_IALG_MemRec m[4];
  TRIK_IALG_Fxns* parent = NULL;
  if (f->ialg.algAlloc(NULL, &parent, m) != 1) return 10;
  void* rec = aligned_alloc(m[0].alignment < 16 ? 16 : m[0].alignment, (m[0].size + 63) / 64 * 64);
  if (!rec) return 11;
  memset(rec, 0xA5, m[0].size);
  m[0].base = rec;
  ((TRIK_IALG_Obj*)rec)->fxns = &f->ialg;
  TRIK_VIDTRANSCODE_CV_Params p;
  memset(&p, 0, sizeof p);
  p.base.size = (int32_t)sizeof p;
  p.base.numOutputStreams = 2;  /* WGLUE:96-101: rejected by setup */
  /* fails on a machine without a HIP device (hipGetDevice) and on one with a
   * device (the params): either way the object is left for algFree */
  int rc = f->ialg.algInit((TRIK_IALG_Handle)rec, m, NULL, (const TRIK_IALG_Params*)&p);
  if (rc == TRIK_IALG_EOK) return 12;
  if (f->ialg.algFree((TRIK_IALG_Handle)rec, m) != 1 || m[0].base != rec) return 13;
  free(rec);
  printf("ok %d\n", rc);
  return 0;
}
"""


def build_xdais_fail(d):
    lib_dir = os.path.join(ROOT, "trik-media-sensors-dsp_amd", "trik_hsv")
    c, exe = os.path.join(d, "xf.c"), os.path.join(d, "xf")
    open(c, "w").write(XDAIS_FAIL_PROG)
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{os.path.join(ROOT, 'include')}", c,
                    f"-L{lib_dir}", "-ltrik_hsv", f"-Wl,-rpath,{lib_dir}", "-o", exe], check=True)
    return exe


def test_xdais_algfree_after_failed_alginit():
    """algInit fails (no HIP device here; rejected params on a GPU box):
    algFree on the record then destroys the object once and returns the
    record, as TI's ALG_create does after a failed algInit."""
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([build_xdais_fail(d)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("ok")
