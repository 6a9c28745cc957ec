/*
 * trik_hsv.h -- C ABI of the MI355X-native TRIK HSV-threshold + centroid path.
 *
 * Drop-in boundary for the reference's object-sensor codec.  All paths below
 * are relative to the reference checkout (trikset/trik-media-sensors-dsp):
 *   WPUB   trik/webcam/object_sensor/trik_vidtranscode_cv.h
 *   OPUB   trik/ov7670/object_sensor/trik_vidtranscode_cv.h
 *   WFXNS  trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c
 *   WGLUE  trik/webcam/object_sensor/src/vidtranscode_cv.cpp
 *   WINT   trik/webcam/object_sensor/include/internal/vidtranscode_cv.h
 *   WSEQ   trik/webcam/object_sensor/include/internal/cv_ball_detector_seqpass.hpp
 *
 * Two layers:
 *  1. The XDAIS-shaped quartet create / control / process / delete.  It keeps
 *     the reference's struct field order, argument meaning and return codes
 *     (TI's xdas.h / ialg.h / xdm.h / ividtranscode.h are not in this image,
 *     so the base structs are restated here with 32-bit XDAS_Int32 fields;
 *     sizes are this ABI's, documented in INTEGRATION.md).  process() takes a
 *     host frame, like the reference's ARM->DSP call.
 *  2. A batched device API (trik_hsv_*) that the quartet sits on: N frames
 *     resident in HBM, T HSV ranges, per-frame per-range results.  This is
 *     where the HIP kernels run.
 *
 * No torch or HIP types cross this ABI: device buffers and streams are plain
 * pointers (a hipStream_t passed as void*; NULL = the null stream).
 * Errors are return codes; no C++ exception crosses it.
 */
#ifndef TRIK_HSV_H_
#define TRIK_HSV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------- */
/* Return codes and XDM constants (TI ialg.h / xdm.h values)               */
/* ---------------------------------------------------------------------- */
#define TRIK_IALG_EOK 0                   /* IALG_EOK */
#define TRIK_IALG_EFAIL (-1)              /* IALG_EFAIL */
#define TRIK_IVIDTRANSCODE_EOK 0          /* IVIDTRANSCODE_EOK */
#define TRIK_IVIDTRANSCODE_EFAIL (-1)     /* IVIDTRANSCODE_EFAIL */
#define TRIK_IVIDTRANSCODE_EUNSUPPORTED (-3) /* IVIDTRANSCODE_EUNSUPPORTED */

/* XDM_CmdId (control commands used at WFXNS:285-330) */
#define TRIK_XDM_GETSTATUS 0
#define TRIK_XDM_SETPARAMS 1
#define TRIK_XDM_RESET 2
#define TRIK_XDM_SETDEFAULT 3
#define TRIK_XDM_FLUSH 4
#define TRIK_XDM_GETBUFINFO 5
#define TRIK_XDM_GETVERSION 6

/* extendedError bits set by XDM_SETUNSUPPORTEDPARAM / XDM_SETCORRUPTEDDATA */
#define TRIK_XDM_CORRUPTEDDATA_BIT 11
#define TRIK_XDM_UNSUPPORTEDPARAM_BIT 14
/* accessMask bits (XDM_SETACCESSMODE_READ / _WRITE) */
#define TRIK_XDM_ACCESSMODE_READ 0
#define TRIK_XDM_ACCESSMODE_WRITE 1

#define TRIK_XDM_CUSTOMENUMBASE 0x100     /* XDM_CUSTOMENUMBASE (TI xdm.h) */
#define TRIK_IVIDTRANSCODE_MAXOUTSTREAMS 2
#define TRIK_XDM_MAX_IO_BUFFERS 16

/* TRIK_VIDTRANSCODE_CV_VideoFormat, WPUB:21-29 and OPUB:21-32 */
typedef enum TRIK_VIDTRANSCODE_CV_VideoFormat {
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_UNKNOWN = 0,
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB888 = TRIK_XDM_CUSTOMENUMBASE,
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB565,
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB565X,
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV444,
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422,  /* packed YUYV (webcam) */
  TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422P  /* Y plane + chroma plane (ov7670) */
} TRIK_VIDTRANSCODE_CV_VideoFormat;

/* ---------------------------------------------------------------------- */
/* XDAIS-mirror structs                                                    */
/* ---------------------------------------------------------------------- */

/* IVIDTRANSCODE_Params, field order from the initialiser at WGLUE:153-184. */
typedef struct TRIK_IVIDTRANSCODE_Params {
  int32_t size;
  int32_t numOutputStreams;
  int32_t formatInput;
  int32_t formatOutput[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t maxHeightInput;
  int32_t maxWidthInput;
  int32_t maxFrameRateInput;
  int32_t maxBitRateInput;
  int32_t maxHeightOutput[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t maxWidthOutput[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t maxFrameRateOutput[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t maxBitRateOutput[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t dataEndianness;
} TRIK_IVIDTRANSCODE_Params;

/* TRIK_VIDTRANSCODE_CV_Params, WPUB:32-34 */
typedef struct TRIK_VIDTRANSCODE_CV_Params {
  TRIK_IVIDTRANSCODE_Params base;
} TRIK_VIDTRANSCODE_CV_Params;

/* IVIDTRANSCODE_DynamicParams, field order from WGLUE:205-258. */
typedef struct TRIK_IVIDTRANSCODE_DynamicParams {
  int32_t size;
  int32_t readHeaderOnlyFlag;
  int32_t keepInputResolutionFlag[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t outputHeight[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t outputWidth[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t keepInputFrameRateFlag[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t inputFrameRate;
  int32_t outputFrameRate[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t targetBitRate[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t rateControl[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t keepInputGOPFlag[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t intraFrameInterval[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t interFrameInterval[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t forceFrame[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t frameSkipTranscodeFlag[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
} TRIK_IVIDTRANSCODE_DynamicParams;

/* TRIK_VIDTRANSCODE_CV_DynamicParams, WPUB:37-45 */
typedef struct TRIK_VIDTRANSCODE_CV_DynamicParams {
  TRIK_IVIDTRANSCODE_DynamicParams base;
  int32_t inputHeight;
  int32_t inputWidth;
  int32_t inputLineLength;
  int32_t outputLineLength[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
} TRIK_VIDTRANSCODE_CV_DynamicParams;

/* TRIK_VIDTRANSCODE_CV_InArgsAlg, WPUB:48-56 (XDAS_Bool restated as int32) */
typedef struct TRIK_VIDTRANSCODE_CV_InArgsAlg {
  uint16_t detectHueFrom; /* [0..359] */
  uint16_t detectHueTo;   /* [0..359]; From > To wraps through 0 (WSEQ:439-445) */
  uint8_t detectSatFrom;  /* [0..100] */
  uint8_t detectSatTo;
  uint8_t detectValFrom;  /* [0..100] */
  uint8_t detectValTo;
  int32_t autoDetectHsv;  /* fill OutArgsAlg.detect* (WSEQ:455-462); detection unchanged */
} TRIK_VIDTRANSCODE_CV_InArgsAlg;

/* IVIDTRANSCODE_InArgs base fields used at WFXNS:192-224 */
typedef struct TRIK_IVIDTRANSCODE_InArgs {
  int32_t size;
  int32_t numBytes;
  int32_t inputID;
} TRIK_IVIDTRANSCODE_InArgs;

typedef struct TRIK_VIDTRANSCODE_CV_InArgs { /* WPUB:58-61 */
  TRIK_IVIDTRANSCODE_InArgs base;
  TRIK_VIDTRANSCODE_CV_InArgsAlg alg;
} TRIK_VIDTRANSCODE_CV_InArgs;

/* TRIK_VIDTRANSCODE_CV_OutArgsAlg, WPUB:64-74 */
typedef struct TRIK_VIDTRANSCODE_CV_OutArgsAlg {
  int8_t targetX;    /* [-100..100] */
  int8_t targetY;    /* [-100..100] */
  uint8_t targetSize; /* [0..100] */
  uint16_t detectHue;
  uint16_t detectHueTolerance;
  uint16_t detectSat;
  uint16_t detectSatTolerance;
  uint16_t detectVal;
  uint16_t detectValTolerance;
} TRIK_VIDTRANSCODE_CV_OutArgsAlg;

/* The ov7670 object sensor's InArgsAlg (OPUB:51-60): a centre and tolerance
 * per channel, applied when setHsvRange is set and kept until the next set
 * (BitmapBuilder, cv_bitmap_builder_reference.hpp:110-130). */
typedef struct TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg {
  int32_t setHsvRange;
  uint16_t detectHue;    /* [0..359] */
  uint16_t detectHueTol; /* [0..359] */
  uint8_t detectSat;     /* [0..100] */
  uint8_t detectSatTol;
  uint8_t detectVal;     /* [0..100] */
  uint8_t detectValTol;
  int32_t autoDetectHsv; /* not reproduced (srand(time) annealing); detect* untouched */
} TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg;

typedef struct TRIK_VIDTRANSCODE_CV_OV7670_InArgs { /* OPUB:62-65 */
  TRIK_IVIDTRANSCODE_InArgs base;
  TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg alg;
} TRIK_VIDTRANSCODE_CV_OV7670_InArgs;

/* XDAS_Target, OPUB:67-71 */
typedef struct TRIK_XDAS_Target {
  int8_t x;     /* [-100..100] */
  int8_t y;     /* [-100..100] */
  uint8_t size; /* [0..100] */
} TRIK_XDAS_Target;

/* The ov7670 object sensor's OutArgsAlg, OPUB:73-81 */
typedef struct TRIK_VIDTRANSCODE_CV_OV7670_OutArgsAlg {
  TRIK_XDAS_Target target[8];
  uint16_t detectHue;
  uint16_t detectHueTolerance;
  uint16_t detectSat;
  uint16_t detectSatTolerance;
  uint16_t detectVal;
  uint16_t detectValTolerance;
} TRIK_VIDTRANSCODE_CV_OV7670_OutArgsAlg;

/* XDM1_SingleBufDesc */
typedef struct TRIK_XDM1_SingleBufDesc {
  int8_t* buf;
  int32_t bufSize;
  int32_t accessMask;
} TRIK_XDM1_SingleBufDesc;

/* XDM1_BufDesc (process input, WFXNS:199-214) */
typedef struct TRIK_XDM1_BufDesc {
  int32_t numBufs;
  TRIK_XDM1_SingleBufDesc descs[TRIK_XDM_MAX_IO_BUFFERS];
} TRIK_XDM1_BufDesc;

/* XDM_BufDesc (process output, WFXNS:200,228-230) */
typedef struct TRIK_XDM_BufDesc {
  int8_t** bufs;
  int32_t numBufs;
  int32_t* bufSizes;
} TRIK_XDM_BufDesc;

/* IVIDTRANSCODE_OutArgs base fields written at WFXNS:195-261 */
typedef struct TRIK_IVIDTRANSCODE_OutArgs {
  int32_t size;
  int32_t extendedError;
  int32_t bitsConsumed;
  int32_t decodedPictureType;
  int32_t decodedPictureStructure;
  int32_t decodedHeight;
  int32_t decodedWidth;
  TRIK_XDM1_SingleBufDesc encodedBuf[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t bitsGenerated[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t encodedPictureType[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t encodedPictureStructure[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t outputID[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t inputFrameSkipTranscodeFlag[TRIK_IVIDTRANSCODE_MAXOUTSTREAMS];
  int32_t outBufsInUseFlag;
} TRIK_IVIDTRANSCODE_OutArgs;

typedef struct TRIK_VIDTRANSCODE_CV_OutArgs { /* WPUB:76-79 */
  TRIK_IVIDTRANSCODE_OutArgs base;
  TRIK_VIDTRANSCODE_CV_OutArgsAlg alg;
} TRIK_VIDTRANSCODE_CV_OutArgs;

typedef struct TRIK_VIDTRANSCODE_CV_OV7670_OutArgs { /* OPUB:83-86 */
  TRIK_IVIDTRANSCODE_OutArgs base;
  TRIK_VIDTRANSCODE_CV_OV7670_OutArgsAlg alg;
} TRIK_VIDTRANSCODE_CV_OV7670_OutArgs;

/* XDM1_AlgBufInfo subset filled by GETSTATUS/GETBUFINFO (WFXNS:287-297) */
typedef struct TRIK_XDM1_AlgBufInfo {
  int32_t minNumInBufs;
  int32_t minNumOutBufs;
  int32_t minInBufSize[TRIK_XDM_MAX_IO_BUFFERS];
  int32_t minOutBufSize[TRIK_XDM_MAX_IO_BUFFERS];
} TRIK_XDM1_AlgBufInfo;

/* IVIDTRANSCODE_Status */
typedef struct TRIK_IVIDTRANSCODE_Status {
  int32_t size;
  int32_t extendedError;
  TRIK_XDM1_SingleBufDesc data;
  TRIK_XDM1_AlgBufInfo bufInfo;
} TRIK_IVIDTRANSCODE_Status;

typedef struct TrikCvHandle* TRIK_VIDTRANSCODE_CV_Handle;

/* ---------------------------------------------------------------------- */
/* Layer 1: XDAIS-shaped quartet                                           */
/* ---------------------------------------------------------------------- */

/* Replaces TRIK_VIDTRANSCODE_CV_alloc + _initObj (WFXNS:85-102, 146-166) as
 * driven by Codec Engine's VIDTRANSCODE_create.  params == NULL takes the
 * defaults of WGLUE:153-184 (YUV422 in, RGB565X out, 640x480 max; the cap is
 * a parameter, not a static buffer size, here).  The handle binds to the
 * calling thread's current HIP device.  Returns IALG_EOK / IALG_EFAIL. */
int32_t TRIK_VIDTRANSCODE_CV_create(const TRIK_VIDTRANSCODE_CV_Params* params,
                                    TRIK_VIDTRANSCODE_CV_Handle* out_handle);

/* The same quartet for the ov7670 line sensor's codec (its own DSP server in
 * the reference: trik/ov7670/line_sensor, LineDetector<YUV422P, RGB565X> of
 * include/internal/cv_line_detector_seqpass.hpp -- LSEQ below).  params ==
 * NULL takes that glue's defaults (YUV422P in, RGB565X out; default dynamic
 * output 240 wide x 320 high as its src/vidtranscode_cv.cpp:214,218).
 * control/process/delete are the functions below; process() then runs
 * LineDetector::run (LSEQ:376-476): V-range detection in columns 5..W-5,
 * cross points over rows H/2..H/2+80, its preview overlays; OutArgs.targetY
 * is the cross size.  autoDetectHsv is ignored (the line sensor's detector is
 * seeded by srand(time(NULL))). */
int32_t TRIK_VIDTRANSCODE_CV_create_line(const TRIK_VIDTRANSCODE_CV_Params* params,
                                         TRIK_VIDTRANSCODE_CV_Handle* out_handle);

/* The quartet for the webcam line sensor's codec (trik/webcam/line_sensor,
 * LineDetector<YUV422, RGB565X> of include/internal/
 * cv_line_detector_seqpass.hpp -- LSEQW).  params == NULL takes the webcam
 * glue's defaults (YUV422 = packed YUYV in, RGB565X out; default dynamic
 * output 240 wide x 320 high).  process() runs LineDetector::run (LSEQW:
 * 330-420): the range (H 0..359, S 0..100, V detectValFrom..detectValTo)
 * over every pixel; when more than 10 pixels match, targetX = ((x - W/2) *
 * 200) / W of the mean column, targetY = 0, targetSize = N * 100 / (W * H);
 * the preview is every pixel (matches white) with magenta lines at columns
 * W/2 +- 40 and +- 80 and a red 3-column line at the mean column.
 * autoDetectHsv is ignored (its detector is seeded by srand(time(NULL))). */
int32_t TRIK_VIDTRANSCODE_CV_create_webcam_line(const TRIK_VIDTRANSCODE_CV_Params* params,
                                                TRIK_VIDTRANSCODE_CV_Handle* out_handle);

/* The quartet for the ov7670 object sensor's codec (trik/ov7670/object_sensor:
 * BallDetector<YUV422P, RGB565X> of include/internal/
 * cv_ball_detector_seqpass.hpp:516-602 -- OSEQ -- with its BitmapBuilder and
 * Clusterizer).  params == NULL takes that glue's defaults (YUV422P in,
 * RGB565X out).  process() then takes TRIK_VIDTRANSCODE_CV_OV7670_InArgs and
 * TRIK_VIDTRANSCODE_CV_OV7670_OutArgs (size fields checked): the sticky HSV
 * range, the 4x4 metapixel bitmap, the clusterer and up to 8 targets by
 * size, and the preview (set metapixels as 0x00ffff, guide lines, a 3x3 red
 * mark per target).  Frames up to 2048x2048 (the reference: 640x480). */
int32_t TRIK_VIDTRANSCODE_CV_create_ov7670(const TRIK_VIDTRANSCODE_CV_Params* params,
                                           TRIK_VIDTRANSCODE_CV_Handle* out_handle);

/* Replaces TRIK_VIDTRANSCODE_CV_free (WFXNS:114-136). */
int32_t TRIK_VIDTRANSCODE_CV_delete(TRIK_VIDTRANSCODE_CV_Handle handle);

/* Replaces TRIK_VIDTRANSCODE_CV_process (WFXNS:174-264).  One host frame in
 * (in_bufs->descs[0]), targetX/Y/Size out in out_args->alg (and detect* when
 * autoDetectHsv is set).  With numOutputStreams == 1 the RGB565X preview is
 * rendered into out_bufs->bufs[0] (see trik_hsv_batch_preview);
 * numOutputStreams == 0 is accepted and writes nothing.  Returns IVIDTRANSCODE_EOK / _EFAIL /
 * _EUNSUPPORTED with the reference's extendedError bits. */
int32_t TRIK_VIDTRANSCODE_CV_process(TRIK_VIDTRANSCODE_CV_Handle handle,
                                     TRIK_XDM1_BufDesc* in_bufs, TRIK_XDM_BufDesc* out_bufs,
                                     TRIK_VIDTRANSCODE_CV_InArgs* in_args,
                                     TRIK_VIDTRANSCODE_CV_OutArgs* out_args);

/* Replaces TRIK_VIDTRANSCODE_CV_control (WFXNS:272-334): GETSTATUS,
 * GETBUFINFO, SETPARAMS (re-runs setup, WGLUE:202-286), RESET/SETDEFAULT,
 * FLUSH, GETVERSION ("1.00.00.00"). */
int32_t TRIK_VIDTRANSCODE_CV_control(TRIK_VIDTRANSCODE_CV_Handle handle, int32_t cmd,
                                     TRIK_VIDTRANSCODE_CV_DynamicParams* dyn_params,
                                     TRIK_IVIDTRANSCODE_Status* status);

/* ---------------------------------------------------------------------- */
/* Layer 1b: the XDAIS function tables (WFXNS:20-66, 85-166)               */
/* ---------------------------------------------------------------------- */
/* What a Codec-Engine-style framework binds: IALG_Fxns + IVIDTRANSCODE_Fxns,
 * restated from TI XDAIS ialg.h / ividtranscode.h (absent here; Int/Uns are
 * 32-bit on the C64x+, so int32_t/uint32_t).  The framework calls algAlloc
 * for the memory records, allocates them, stores the table in the object's
 * first word (IALG_Obj.fxns), calls algInit, then process/control through
 * the table, then algFree and releases the records.  The object IS a
 * TRIK_VIDTRANSCODE_CV_Handle: the table's process/control are the quartet's
 * process/control, and TRIK_VIDTRANSCODE_CV_create/_delete are the same
 * alloc + init / free with the library owning the memory. */
typedef enum TRIK_IALG_MemAttrs { TRIK_IALG_SCRATCH = 0, TRIK_IALG_PERSIST = 1, TRIK_IALG_WRITEONCE = 2 } TRIK_IALG_MemAttrs;
#define TRIK_IALG_MXTRN 0x0010 /* ialg.h: external memory space bit */
#define TRIK_IALG_DARAM0 0
#define TRIK_IALG_EXTERNAL (TRIK_IALG_MXTRN + 1)

typedef struct TRIK_IALG_MemRec {
  uint32_t size;      /* Uns */
  int32_t alignment;  /* Int: 0 = any */
  int32_t space;      /* IALG_MemSpace */
  int32_t attrs;      /* IALG_MemAttrs */
  void* base;
} TRIK_IALG_MemRec;

struct TRIK_IALG_Fxns;
typedef struct TRIK_IALG_Obj {
  const struct TRIK_IALG_Fxns* fxns;
} TRIK_IALG_Obj;
typedef TRIK_IALG_Obj* TRIK_IALG_Handle;

/* IALG_Params: the codec's TRIK_VIDTRANSCODE_CV_Params (its first field is the size). */
typedef struct TRIK_IALG_Params {
  int32_t size;
} TRIK_IALG_Params;

typedef struct TRIK_IALG_Fxns {
  const void* implementationId;
  void (*algActivate)(TRIK_IALG_Handle);
  int32_t (*algAlloc)(const TRIK_IALG_Params*, struct TRIK_IALG_Fxns**, TRIK_IALG_MemRec*);
  int32_t (*algControl)(TRIK_IALG_Handle, int32_t, void*);
  void (*algDeactivate)(TRIK_IALG_Handle);
  int32_t (*algFree)(TRIK_IALG_Handle, TRIK_IALG_MemRec*);
  int32_t (*algInit)(TRIK_IALG_Handle, const TRIK_IALG_MemRec*, TRIK_IALG_Handle, const TRIK_IALG_Params*);
  void (*algMoved)(TRIK_IALG_Handle, const TRIK_IALG_MemRec*, TRIK_IALG_Handle, const TRIK_IALG_Params*);
  int32_t (*algNumAlloc)(void);
} TRIK_IALG_Fxns;

/* IVIDTRANSCODE_Fxns.  in_args / out_args: the codec's InArgs / OutArgs
 * (size fields checked), as IVIDTRANSCODE_InArgs* / _OutArgs* in TI's. */
typedef struct TRIK_IVIDTRANSCODE_Fxns {
  TRIK_IALG_Fxns ialg;
  int32_t (*process)(TRIK_IALG_Handle, TRIK_XDM1_BufDesc*, TRIK_XDM_BufDesc*, TRIK_IVIDTRANSCODE_InArgs*,
                     TRIK_IVIDTRANSCODE_OutArgs*);
  int32_t (*control)(TRIK_IALG_Handle, int32_t, TRIK_VIDTRANSCODE_CV_DynamicParams*, TRIK_IVIDTRANSCODE_Status*);
} TRIK_IVIDTRANSCODE_Fxns;

/* The webcam object sensor's tables (WFXNS:36-66); IALG is the same table
 * as FXNS.ialg (the reference aliases the two symbols on TI toolchains and
 * duplicates them elsewhere, as here).  The other three codecs of this library
 * (one DSP server each in the reference, all named TRIK_VIDTRANSCODE_CV_FXNS
 * there): the ov7670 object sensor, the ov7670 line sensor and the webcam
 * line sensor. */
extern TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_FXNS;
extern TRIK_IALG_Fxns TRIK_VIDTRANSCODE_CV_IALG;
extern TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_OV7670_FXNS;
extern TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_LINE_FXNS;
extern TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_WEBCAM_LINE_FXNS;

/* The webcam object sensor's IALG functions (WFXNS:85-166), also reachable
 * through the tables.  alloc asks for one persistent external record (the
 * object; the reference's second record is C64x+ on-chip fast RAM, which
 * has no use here) and returns the record count; initObj constructs the
 * object in that record (keeping the framework's fxns word) and runs the
 * setup of WFXNS:146-166; free destroys it and returns the record for the
 * framework to release. */
int32_t TRIK_VIDTRANSCODE_CV_alloc(const TRIK_IALG_Params* params, TRIK_IALG_Fxns** parent_fxns,
                                   TRIK_IALG_MemRec mem_tab[]);
int32_t TRIK_VIDTRANSCODE_CV_initObj(TRIK_IALG_Handle handle, const TRIK_IALG_MemRec mem_tab[],
                                     TRIK_IALG_Handle parent, const TRIK_IALG_Params* params);
int32_t TRIK_VIDTRANSCODE_CV_free(TRIK_IALG_Handle handle, TRIK_IALG_MemRec mem_tab[]);

/* ---------------------------------------------------------------------- */
/* Layer 2: batched device API                                             */
/* ---------------------------------------------------------------------- */

#define TRIK_HSV_LAYOUT_YUYV 0   /* packed Y0 U Y1 V, row = 2*W bytes (WSEQ:251-284) */
#define TRIK_HSV_LAYOUT_OV7670 1 /* Y plane rows + chroma plane rows; U = odd, V = even
                                    chroma byte (OSEQ:343-387) */

/* N frames in device memory: frame i starts at frames + i * frame_stride.
 * One frame is height * line_length bytes (YUYV) or 2 * height * line_length
 * (ov7670, chroma plane right after the luma plane).  Geometry rules of
 * WSEQ:365-369: width % 32 == 0, height % 4 == 0, both >= 0; line_length >=
 * 2*width (YUYV) or >= width (ov7670). */
typedef struct TrikHsvFrameBatch {
  const void* frames;
  int64_t frame_stride;
  int32_t n_frames;
  int32_t width;
  int32_t height;
  int32_t line_length;
  int32_t layout;
} TrikHsvFrameBatch;

/* Per frame per range: the reference's m_targetPoints / m_targetX / m_targetY
 * (WSEQ:56-58, accumulated at WSEQ:350-352), widened to 64 bits. */
typedef struct TrikHsvTargetSums {
  int64_t points;
  int64_t sum_x;
  int64_t sum_y;
} TrikHsvTargetSums;

/* Per frame per range: OutArgsAlg.targetX/targetY/targetSize (WSEQ:486-505). */
typedef struct TrikHsvTarget {
  int8_t x;
  int8_t y;
  uint8_t size;
  uint8_t reserved;
} TrikHsvTarget;

#define TRIK_HSV_MAX_RANGES 64

const char* trik_hsv_version(void);
/* Message of the last failed call on this thread ("" if none). */
const char* trik_hsv_last_error(void);

/* Full batched process: zero sums, detect + reduce, epilogue.
 * sums_dev: [n_frames][n_ranges] TrikHsvTargetSums (device).
 * targets_dev: [n_frames][n_ranges] TrikHsvTarget (device) or NULL.
 * Returns 0 or TRIK_IVIDTRANSCODE_EFAIL (see trik_hsv_last_error()). */
int32_t trik_hsv_process_batch(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                               const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n_ranges,
                               TrikHsvTargetSums* sums_dev, TrikHsvTarget* targets_dev,
                               void* hip_stream);

/* The full batched step: as trik_hsv_process_batch, plus the per-target
 * batch totals (totals_dev[r] = the sum over the frames of sums_dev[f][r], as
 * trik_hsv_batch_totals).  Where the chroma-run kernel runs, each group of
 * <= 4 ranges is ONE launch: the kernel writes every frame's sums and targets
 * as the frame completes and the totals at its end (scratch held by the
 * handle); otherwise the same outputs come from the separate kernels.
 * totals_dev: [n_ranges] TrikHsvTargetSums (device, not NULL). */
int32_t trik_hsv_process_batch_totals(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                                      const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n_ranges,
                                      TrikHsvTargetSums* sums_dev, TrikHsvTarget* targets_dev,
                                      TrikHsvTargetSums* totals_dev, void* hip_stream);

/* Detect + reduce only; ADDS into sums_dev (caller zeroes it).  This is the
 * hot kernel, one launch per group of <= 4 ranges. */
int32_t trik_hsv_batch_sums(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                            const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n_ranges,
                            TrikHsvTargetSums* sums_dev, void* hip_stream);

/* Hot-kernel selection of one handle for its trik_hsv_batch_sums /
 * _process_batch / _masks / _blob_batch calls and process() (tests and A/B
 * runs; other handles are not affected).  TRIK_HSV_HOT_AUTO (the default)
 * picks, per group of 4 ranges, the chroma-run kernel for batches of at
 * least TRIK_HSV_CHROMA_MIN_PIXELS pixels whose geometry it takes when the
 * group's tables send at most TRIK_HSV_CHROMA_MAX_SHARE of the words to its
 * exact path (see trik_hsv_chroma_share), the stripe kernel otherwise -- always for a
 * group of ranges that accepts every hue and saturation (value bands), which
 * the stripe kernel tests by value alone; all kernels give the same results.
 * The first batch with a new range set is not held up by that
 * share: both kernels are enqueued and the device runs the one the rule picks.
 * Returns the previous setting, or -1 for a NULL handle or an unknown kind. */
#define TRIK_HSV_HOT_AUTO 0
#define TRIK_HSV_HOT_STRIPE 1
#define TRIK_HSV_HOT_CHROMA 2
#define TRIK_HSV_HOT_GENERIC 3
#define TRIK_HSV_HOT_MIXED 4 /* trik_hsv_last_hot_kernel: the call's range groups ran different kernels */
#define TRIK_HSV_CHROMA_MIN_PIXELS (32 * 640 * 480)
#define TRIK_HSV_CHROMA_MAX_SHARE 0.27 /* the measured crossover (profiles/r05/r05p_adversarial_4096.txt) */
int32_t trik_hsv_set_hot_kernel(TRIK_VIDTRANSCODE_CV_Handle handle, int32_t kind);
/* The chroma-run kernel's expected exact-path word share (uniform input) for
 * the handle's current batched-sums range set (the maximum over its groups of
 * 4 ranges), or -1 when its tables are not built.  Waits for the builder's
 * readback if it is still in flight.  Returns 0 or TRIK_IVIDTRANSCODE_EFAIL. */
int32_t trik_hsv_chroma_share(TRIK_VIDTRANSCODE_CV_Handle handle, double* share);
/* The share of words the chroma-run kernel's exact path actually resolved on
 * the handle's recent batches of that range set that ran it (the maximum over
 * its groups; -1 before two readbacks have landed; intervals with a batch on
 * which the device chose the kernel are not measured).  AUTO reads the kernel's
 * counter back every few launches without waiting and sends a group whose
 * measured share exceeds TRIK_HSV_CHROMA_MAX_SHARE -- input concentrated on
 * the chromas its tables describe worst -- to the stripe kernel, trying the
 * chroma-run kernel again every 32 batches.  Waits for a readback in flight. */
int32_t trik_hsv_chroma_measured_share(TRIK_VIDTRANSCODE_CV_Handle handle, double* share);
/* The kernel the handle's last hot call ran (TRIK_HSV_HOT_STRIPE, _CHROMA or
 * _GENERIC; TRIK_HSV_HOT_MIXED when its groups of 4 ranges ran different
 * kernels; 0 before any; a call with an empty batch launches nothing and
 * leaves the answer unchanged).  When the device chose (see above) this waits for
 * the builder's readback. */
int32_t trik_hsv_last_hot_kernel(TRIK_VIDTRANSCODE_CV_Handle handle);
/* CUs the chroma-run hot kernel leaves free (0 by default): its grid is one
 * 160-KiB-LDS workgroup per CU the stream may use, so a kernel on another
 * stream (the per-step all-reduce of the totals over RCCL, multi-GPU) waits
 * for a CU to free up unless some stay free.  n CUs fewer: ~n/256 slower at
 * MI355X's 256 CUs; results are identical.  0 <= n <= 32; returns the
 * previous setting, or -1 for a NULL handle or an n out of range.  A stream
 * created with a CU mask (hipExtStreamCreateWithCUMask) is sized to its mask
 * where the runtime reports it. */
int32_t trik_hsv_set_reserved_cus(TRIK_VIDTRANSCODE_CV_Handle handle, int32_t n);

/* Epilogue only: sums_dev -> targets_dev for an n_frames x n_ranges grid. */
int32_t trik_hsv_batch_targets(const TrikHsvFrameBatch* batch, int32_t n_ranges,
                               const TrikHsvTargetSums* sums_dev, TrikHsvTarget* targets_dev,
                               void* hip_stream);

/* Verification mode of the hot kernel: also writes the per-pixel detection
 * mask (bit t = range t, n_ranges <= 8) to masks_dev[n_frames][height][width]
 * and adds into sums_dev.  Not used on the timed path. */
int32_t trik_hsv_batch_masks(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                             const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n_ranges,
                             uint8_t* masks_dev, TrikHsvTargetSums* sums_dev, void* hip_stream);

/* The operator's preview stream for N frames and one range (SURVEY 8(f)
 * row 2): each preview (out_height rows of out_line_length bytes at
 * previews_dev + i * preview_stride) is zero-filled (WFXNS:234), then written
 * as proceedImageHsv does -- RGB565X (B5 G6 R5, R in the low bits) of every
 * source pixel through the truncated scale maps, last writer wins, detected
 * pixels as 0x00ffff (WSEQ:316-354, 371-387) -- and overlaid with the guide
 * lines and the target circle (WSEQ:66-166, 471-494).  The circle uses
 * sums_dev[i * sums_pitch] (this range's sums of frame i, e.g. from
 * trik_hsv_process_batch with sums_pitch = n_ranges). */
int32_t trik_hsv_batch_preview(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                               const TRIK_VIDTRANSCODE_CV_InArgsAlg* range,
                               const TrikHsvTargetSums* sums_dev, int32_t sums_pitch,
                               int32_t out_width, int32_t out_height, int32_t out_line_length,
                               uint8_t* previews_dev, int64_t preview_stride, void* hip_stream);

/* autoDetectHsv for N frames: HsvRangeDetector::detect
 * (trik/webcam/object_sensor/include/internal/cv_hsv_range_detector.hpp:
 * 88-198, zone scale 6 as WSEQ:32).  out_dev[i][6] = detectHue,
 * detectHueTolerance, detectSat, detectSatTolerance, detectVal,
 * detectValTolerance (uint16), as OutArgsAlg receives them. */
int32_t trik_hsv_batch_auto_range(const TrikHsvFrameBatch* batch, uint16_t* out_dev, void* hip_stream);

/* The line sensor for N ov7670 frames: sums_dev[i] =
 * {points, sum_x, cross points} -- cross points in the sum_y slot -- for V in
 * [val_from, val_to] (InArgs percent units) in columns 5..W-5, cross points
 * over rows band_start..band_stop (the reference: H/2 .. H/2+80);
 * targets_dev[i] (may be NULL) = OutArgs of LSEQ:455-474. */
int32_t trik_hsv_line_batch(const TrikHsvFrameBatch* batch, int32_t val_from, int32_t val_to,
                            int32_t band_start, int32_t band_stop, TrikHsvTargetSums* sums_dev,
                            TrikHsvTarget* targets_dev, void* hip_stream);

/* The line sensor's preview for N frames (window columns, guide, band and
 * target lines, LSEQ:283-291, 433-467), from sums_dev of trik_hsv_line_batch. */
int32_t trik_hsv_line_preview(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                              int32_t val_from, int32_t val_to, const TrikHsvTargetSums* sums_dev,
                              int32_t out_width, int32_t out_height, int32_t out_line_length,
                              uint8_t* previews_dev, int64_t preview_stride, void* hip_stream);

/* The ov7670 multi-blob sensor for N ov7670 frames,
 * one HSV range given as the InArgs centre/tolerance (converted as
 * cv_bitmap_builder_reference.hpp:110-130):
 *   targets_dev  [N][8] TrikHsvTarget: OutArgs target[i] (x, y, size; 0 when
 *                not kept), OSEQ:563-590;
 *   top_dev      optional [N][8][3] int32: size, sum_x, sum_y of the 8
 *                largest clusters after the clusterer's postProcessing;
 *   meta_dev     optional [N][H/4][W/4] uint8: 1 for set metapixels (more than
 *                2 of 16 pixels detected);
 *   labels_dev   optional [N][H/4][W/4] uint16: the clusterer's label map;
 *   n_labels_dev optional [N] int32: labels including the background.
 * Scratch lives in the handle. */
int32_t trik_hsv_blob_batch(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                            const TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg* hsv, TrikHsvTarget* targets_dev,
                            int32_t* top_dev, uint8_t* meta_dev, uint16_t* labels_dev,
                            int32_t* n_labels_dev, void* hip_stream);

/* Its previews for N frames from meta_dev and top_dev of trik_hsv_blob_batch
 * (OSEQ:387-420, 548-580). */
int32_t trik_hsv_blob_preview(TRIK_VIDTRANSCODE_CV_Handle handle, const TrikHsvFrameBatch* batch,
                              const uint8_t* meta_dev, const int32_t* top_dev, int32_t out_width,
                              int32_t out_height, int32_t out_line_length, uint8_t* previews_dev,
                              int64_t preview_stride, void* hip_stream);

/* Fill batch->frames (device, writable) with synthetic frames; frame i of the
 * batch is global frame first_frame + i.  kind 0 = uniform random bytes,
 * kind 1 = scene (gradients + 6 coloured discs).  Same bytes as the CPU
 * generator in oracle/trik_oracle.c for the same (seed, frame). */
int32_t trik_hsv_synth(const TrikHsvFrameBatch* batch, int32_t first_frame, int32_t kind,
                       uint64_t seed, void* hip_stream);

/* ---------------------------------------------------------------------- */
/* Layer 3: multi-GPU                                        */
/* ---------------------------------------------------------------------- */
/* Frames are independent units: a batch is sharded by frame index, each GPU
 * processes its shard resident in its own memory, and the one exchange is the
 * sum of the per-target batch totals (n_ranges x 3 int64) with one RCCL
 * all-reduce over xGMI.  The reference has no multi-device path (one DSP, one
 * frame per process call, WFXNS:174-264); these extend its batched surface.
 * RCCL (librccl.so.1) is loaded on the first group/comm call. */

/* Per-target batch totals on the device: totals_dev[r] = the sum over the
 * n_frames frames of sums_dev[f][r] (each field), stream-ordered. */
int32_t trik_hsv_batch_totals(int32_t n_frames, int32_t n_ranges, const TrikHsvTargetSums* sums_dev,
                              TrikHsvTargetSums* totals_dev, void* hip_stream);

/* One process driving several GPUs: per device an object-sensor handle
 * (TRIK_VIDTRANSCODE_CV_create defaults), a HIP stream and a host worker
 * thread, and an RCCL communicator over the devices (ncclCommInitAll). */
typedef struct TrikHsvGroup* TRIK_HSV_GroupHandle;
int32_t trik_hsv_group_create(int32_t n_devices, const int32_t* devices, TRIK_HSV_GroupHandle* out_group);
/* Device d (0 <= d < n_devices) processes batches[d] -- its frames, in the
 * memory of devices[d] -- as trik_hsv_process_batch does into sums_dev[d]
 * ([n_frames][n_ranges]) and targets_dev[d] (may be NULL), then the per-target
 * totals of its frames are summed over all devices with one ncclAllReduce
 * into totals_dev[d] ([n_ranges], on devices[d]), so every device holds the
 * totals of the whole batch.  Each device's worker thread enqueues its part on
 * the device's stream; the call returns once every part is enqueued (see
 * trik_hsv_group_sync).  A device with an empty shard (n_frames == 0) still
 * takes part in the all-reduce. */
int32_t trik_hsv_group_process(TRIK_HSV_GroupHandle group, const TrikHsvFrameBatch* batches,
                               const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n_ranges,
                               TrikHsvTargetSums* const* sums_dev, TrikHsvTarget* const* targets_dev,
                               TrikHsvTargetSums* const* totals_dev);
/* Waits for every device's enqueued work. */
int32_t trik_hsv_group_sync(TRIK_HSV_GroupHandle group);
/* The HIP stream device d's work runs on (for the caller's own ordering). */
void* trik_hsv_group_stream(TRIK_HSV_GroupHandle group, int32_t d);
int32_t trik_hsv_group_delete(TRIK_HSV_GroupHandle group);

/* One process per GPU (the layout of torch.distributed / bench.py): an RCCL
 * communicator over n_ranks processes, created on the calling thread's current
 * device from an id that rank 0 makes (trik_hsv_comm_id) and the caller
 * distributes to the other ranks by its own means. */
#define TRIK_HSV_COMM_ID_BYTES 128
typedef struct TrikHsvComm* TRIK_HSV_CommHandle;
int32_t trik_hsv_comm_id(uint8_t id[TRIK_HSV_COMM_ID_BYTES]);
int32_t trik_hsv_comm_create(int32_t n_ranks, int32_t rank, const uint8_t id[TRIK_HSV_COMM_ID_BYTES],
                             TRIK_HSV_CommHandle* out_comm);
/* In place, stream-ordered: totals_dev[n_ranges] summed over the ranks. */
int32_t trik_hsv_comm_all_reduce_totals(TRIK_HSV_CommHandle comm, TrikHsvTargetSums* totals_dev,
                                        int32_t n_ranges, void* hip_stream);
int32_t trik_hsv_comm_delete(TRIK_HSV_CommHandle comm);

#ifdef __cplusplus
}
#endif

#endif /* TRIK_HSV_H_ */
