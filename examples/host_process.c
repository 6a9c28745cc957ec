/*
 * host_process.c -- the reference's ARM-side call sequence (Codec Engine
 * VIDTRANSCODE_create / _control / _process / _delete on the object sensor,
 * trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c) made against
 * libtrik_hsv.so in plain C, as INTEGRATION.md section 3 describes.  Like
 * Codec Engine, it binds only the codec's function table
 * (TRIK_VIDTRANSCODE_CV_FXNS, WFXNS:36-40): algAlloc -> allocate the memory
 * records -> algInit -> control / process -> algFree -> release the records
 * (ALG_create / ALG_delete of TI's framework, restated below).
 *
 * usage: host_process FRAME.yuyv WIDTH HEIGHT HUE_FROM HUE_TO SAT_FROM SAT_TO VAL_FROM VAL_TO
 * Reads one packed YUYV frame (lineLength = 2*WIDTH), prints
 *   "rc targetX targetY targetSize preview_crc32"
 * and exits with the process() return code.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "trik_hsv.h"

static uint32_t crc32(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) {
    c ^= p[i];
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return ~c;
}

#define MAX_RECS 16

/* ALG_create: the codec's memory records allocated as it asks, the table in
 * the object's first word, then algInit. */
static TRIK_IALG_Handle alg_create(const TRIK_IVIDTRANSCODE_Fxns* fx, const TRIK_VIDTRANSCODE_CV_Params* params,
                                   TRIK_IALG_MemRec* mem, int* n) {
  TRIK_IALG_Fxns* parent = NULL;
  *n = fx->ialg.algAlloc((const TRIK_IALG_Params*)params, &parent, mem);
  if (*n < 1 || *n > MAX_RECS) return NULL;
  for (int i = 0; i < *n; ++i) {
    size_t align = mem[i].alignment > 16 ? (size_t)mem[i].alignment : 16;
    size_t size = ((size_t)mem[i].size + align - 1) / align * align;
    mem[i].base = aligned_alloc(align, size);
    if (!mem[i].base) return NULL;
    memset(mem[i].base, 0, size);
  }
  TRIK_IALG_Handle alg = (TRIK_IALG_Handle)mem[0].base;
  alg->fxns = &fx->ialg;
  if (fx->ialg.algInit(alg, mem, NULL, (const TRIK_IALG_Params*)params) != TRIK_IALG_EOK) {
    for (int i = 0; i < *n; ++i) free(mem[i].base);
    return NULL;
  }
  return alg;
}

/* ALG_delete: algFree hands back the records, which are released. */
static void alg_delete(const TRIK_IVIDTRANSCODE_Fxns* fx, TRIK_IALG_Handle alg) {
  TRIK_IALG_MemRec mem[MAX_RECS];
  const int n = fx->ialg.algFree(alg, mem);
  for (int i = 0; i < n && i < MAX_RECS; ++i) free(mem[i].base);
}

int main(int argc, char** argv) {
  if (argc != 10) {
    fprintf(stderr, "usage: %s FRAME W H hueFrom hueTo satFrom satTo valFrom valTo\n", argv[0]);
    return 2;
  }
  const int w = atoi(argv[2]), h = atoi(argv[3]), ll = 2 * w;
  const size_t frame_bytes = (size_t)h * (size_t)ll;
  uint8_t* frame = (uint8_t*)malloc(frame_bytes ? frame_bytes : 1);
  FILE* f = fopen(argv[1], "rb");
  if (!frame || !f || fread(frame, 1, frame_bytes, f) != frame_bytes) {
    fprintf(stderr, "cannot read %zu bytes from %s\n", frame_bytes, argv[1]);
    return 2;
  }
  fclose(f);

  const TRIK_IVIDTRANSCODE_Fxns* fx = &TRIK_VIDTRANSCODE_CV_FXNS;
  TRIK_IALG_MemRec mem[MAX_RECS];
  int n_recs = 0;
  TRIK_IALG_Handle hd = alg_create(fx, NULL, mem, &n_recs);  /* VIDTRANSCODE_create */
  if (!hd) {
    fprintf(stderr, "create: %s\n", trik_hsv_last_error());
    return 3;
  }
  TRIK_VIDTRANSCODE_CV_DynamicParams dyn;
  memset(&dyn, 0, sizeof dyn);
  dyn.base.size = sizeof dyn;
  dyn.inputWidth = w;
  dyn.inputHeight = h;
  dyn.inputLineLength = ll;
  dyn.base.outputWidth[0] = w / 2;
  dyn.base.outputHeight[0] = h / 2;
  dyn.outputLineLength[0] = w;  /* RGB565X: 2 bytes per pixel */
  TRIK_IVIDTRANSCODE_Status st;
  memset(&st, 0, sizeof st);
  st.size = sizeof st;
  if (fx->control(hd, TRIK_XDM_SETPARAMS, &dyn, &st) != TRIK_IALG_EOK) {  /* _control */
    fprintf(stderr, "control: %s\n", trik_hsv_last_error());
    return 3;
  }
  const size_t preview_bytes = (size_t)(h / 2) * (size_t)w;
  uint8_t* preview = (uint8_t*)calloc(preview_bytes ? preview_bytes : 1, 1);
  TRIK_XDM1_BufDesc in;
  memset(&in, 0, sizeof in);
  in.numBufs = 1;
  in.descs[0].buf = (int8_t*)frame;
  in.descs[0].bufSize = (int32_t)frame_bytes;
  int8_t* out_buf = (int8_t*)preview;
  int32_t out_size = (int32_t)preview_bytes;
  TRIK_XDM_BufDesc out = {&out_buf, 1, &out_size};
  TRIK_VIDTRANSCODE_CV_InArgs ia;
  memset(&ia, 0, sizeof ia);
  ia.base.size = sizeof ia;
  ia.base.numBytes = (int32_t)frame_bytes;
  ia.alg.detectHueFrom = (uint16_t)atoi(argv[4]);
  ia.alg.detectHueTo = (uint16_t)atoi(argv[5]);
  ia.alg.detectSatFrom = (uint8_t)atoi(argv[6]);
  ia.alg.detectSatTo = (uint8_t)atoi(argv[7]);
  ia.alg.detectValFrom = (uint8_t)atoi(argv[8]);
  ia.alg.detectValTo = (uint8_t)atoi(argv[9]);
  TRIK_VIDTRANSCODE_CV_OutArgs oa;
  memset(&oa, 0, sizeof oa);
  oa.base.size = sizeof oa;
  const int32_t rc = fx->process(hd, &in, &out, (TRIK_IVIDTRANSCODE_InArgs*)&ia,
                                 (TRIK_IVIDTRANSCODE_OutArgs*)&oa);  /* _process */
  printf("%d %d %d %u %08x\n", rc, oa.alg.targetX, oa.alg.targetY, oa.alg.targetSize,
         crc32(preview, preview_bytes));
  alg_delete(fx, hd);  /* VIDTRANSCODE_delete */
  free(preview);
  free(frame);
  return rc == TRIK_IVIDTRANSCODE_EOK ? 0 : 1;
}
