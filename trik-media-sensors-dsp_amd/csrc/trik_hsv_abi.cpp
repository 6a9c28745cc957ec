// trik_hsv_abi.cpp -- C ABI of libtrik_hsv.so (declared in include/trik_hsv.h).
//
// Layer 1 restates the reference's XDAIS codec shell and handle glue:
//   WFXNS trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c
//   WGLUE trik/webcam/object_sensor/src/vidtranscode_cv.cpp
// with per-handle state (the reference keeps its image buffers and LUT
// pointers in process-wide statics, WSEQ:23-26,63-64) and the pixel work on
// the GPU.  Layer 2 (trik_hsv_*) is the batched device API the GPU work sits
// behind.  No C++ exception escapes any entry point.
#include <atomic>
#include <hip/hip_runtime.h>
#include <limits.h>
#include <string.h>

#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "trik_hsv_internal.h"

using namespace trik_hsv;

namespace {

thread_local std::string g_last_error;

int32_t fail(int32_t code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

}  // namespace

// The last-error slot of the calling thread, for the other translation units
// (trik_hsv_group.cpp reports its workers' errors on the caller's thread).
int32_t trik_hsv::set_error(int32_t code, const std::string& msg) { return fail(code, msg); }

namespace {

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (hipError_t)(expr);                                                \
    if (e_ != hipSuccess)                                                              \
      return fail(TRIK_IVIDTRANSCODE_EFAIL, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

const char k_version[] = "1.00.00.00";  // WFXNS:75

const TRIK_VIDTRANSCODE_CV_Params k_default_params = {{
    (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_Params),  // WGLUE:153-184
    1,
    TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422,
    {TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB565X, TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_UNKNOWN},
    480, 640, 60000, -1,
    {480, -1},
    {640, -1},
    {-1, -1},
    {-1, -1},
    1 /* XDM_BYTE */}};

// The algorithms behind a handle: the object sensor (BallDetector, webcam
// WSEQ and ov7670 OSEQ layouts) or the ov7670 line sensor (LineDetector,
// LSEQ = trik/ov7670/line_sensor/include/internal/cv_line_detector_seqpass.hpp;
// its glue trik/ov7670/line_sensor/src/vidtranscode_cv.cpp is WGLUE with
// YUV422P input and a 240x320 default output).
// kAlgoWLine: the webcam line sensor (LineDetector<YUV422, RGB565X> of
// trik/webcam/line_sensor/include/internal/cv_line_detector_seqpass.hpp --
// LSEQW -- with the webcam glue, a 240x320 default output as the line glues).
enum Algo { kAlgoBall = 0, kAlgoLine = 1, kAlgoBlob = 2, kAlgoWLine = 3 };

// ov7670 object sensor glue: the webcam glue with formatInput = YUV422P
// (trik/ov7670/object_sensor/src/vidtranscode_cv.cpp:80,157)
const TRIK_VIDTRANSCODE_CV_Params k_default_params_blob = {{
    (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_Params),
    1,
    TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422P,
    {TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB565X, TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_UNKNOWN},
    480, 640, 60000, -1,
    {480, -1},
    {640, -1},
    {-1, -1},
    {-1, -1},
    1 /* XDM_BYTE */}};

const TRIK_VIDTRANSCODE_CV_Params k_default_params_line = {{
    (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_Params),  // line glue :153-184
    1,
    TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422P,
    {TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB565X, TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_UNKNOWN},
    480, 640, 60000, -1,
    {480, -1},
    {640, -1},
    {-1, -1},
    {-1, -1},
    1 /* XDM_BYTE */}};

TRIK_VIDTRANSCODE_CV_DynamicParams default_dynamic_params(int algo) {  // WGLUE:205-266
  TRIK_VIDTRANSCODE_CV_DynamicParams d;
  memset(&d, 0, sizeof d);
  d.base.size = (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_DynamicParams);
  d.base.readHeaderOnlyFlag = 0;
  d.base.keepInputResolutionFlag[0] = 0;
  d.base.keepInputResolutionFlag[1] = 1;
  const bool line = algo == kAlgoLine || algo == kAlgoWLine;
  d.base.outputHeight[0] = line ? 320 : 240;  // the line glues (:214,218) swap them
  d.base.outputWidth[0] = line ? 240 : 320;
  d.base.keepInputFrameRateFlag[0] = d.base.keepInputFrameRateFlag[1] = 1;
  d.base.inputFrameRate = -1;
  d.base.outputFrameRate[0] = d.base.outputFrameRate[1] = -1;
  d.base.targetBitRate[0] = d.base.targetBitRate[1] = -1;
  d.base.keepInputGOPFlag[0] = d.base.keepInputGOPFlag[1] = 1;
  d.base.intraFrameInterval[0] = d.base.intraFrameInterval[1] = 1;
  d.base.forceFrame[0] = d.base.forceFrame[1] = -1;  // IVIDEO_NA_FRAME
  d.inputHeight = -1;
  d.inputWidth = -1;
  d.inputLineLength = -1;
  d.outputLineLength[0] = d.outputLineLength[1] = -1;
  return d;
}

std::string validate_batch(const TrikHsvFrameBatch* b) {
  if (!b) return "batch is NULL";
  if (b->n_frames < 0) return "n_frames < 0";
  if (b->width < 0 || b->height < 0 || b->width % 32 != 0 || b->height % 4 != 0)
    return "geometry: need width % 32 == 0, height % 4 == 0, both >= 0 (WSEQ:365-369)";
  if (b->width > 32767 || b->height > 32767) return "geometry: width/height exceed int16 (WINT:32)";
  if (b->layout != TRIK_HSV_LAYOUT_YUYV && b->layout != TRIK_HSV_LAYOUT_OV7670) return "unknown layout";
  const int64_t row = b->layout == TRIK_HSV_LAYOUT_YUYV ? 2LL * b->width : (int64_t)b->width;
  if (b->height > 0 && b->line_length < row) return "line_length shorter than a row";
  const int64_t fb = (int64_t)b->height * b->line_length * (b->layout == TRIK_HSV_LAYOUT_OV7670 ? 2 : 1);
  if (b->n_frames > 1 && b->frame_stride < fb) return "frame_stride shorter than a frame";
  if (b->n_frames > 0 && fb > 0 && !b->frames) return "frames is NULL";
  return "";
}

}  // namespace

// ---------------------------------------------------------------------------
// Handle
// ---------------------------------------------------------------------------
// Device buffers a handle shares between calls that may run on different
// streams: the last use on each stream is an event, so that a later call can
// make its stream wait for them (device side) or, before the buffer is
// rewritten, find out without blocking whether they have finished.
// One event per stream the handle has enqueued work on, recorded once per
// call after its last launch (an event record is a packet on the stream: one
// per call, not one per buffer).  A new stream takes over the event of one whose recorded work has
// completed once kMaxMarks streams are tracked, so the list stays bounded
// however many short-lived streams a caller cycles through.
constexpr size_t kMaxMarks = 16;
struct StreamMarks {
  std::vector<std::pair<hipStream_t, hipEvent_t>> marks;
  int32_t mark(hipStream_t s, hipEvent_t* out) {
    std::pair<hipStream_t, hipEvent_t>* slot = nullptr;
    for (auto& m : marks)
      if (m.first == s) {
        slot = &m;
        break;
      }
    if (!slot && marks.size() >= kMaxMarks)
      for (auto& m : marks)
        if (hipEventQuery(m.second) == hipSuccess) {
          m.first = s;
          slot = &m;
          break;
        }
    if (!slot) {
      hipEvent_t e = nullptr;
      // device-scope release, no system-scope fence: the marks order streams
      // of this device and tell the host that work has finished; none makes
      // device writes visible to the host (callers' copies do that).  With
      // the default system-scope fence a record cost ~5.7 us between two
      // back-to-back steps (L2 written back and invalidated:
      // profiles/r04/r04k_driver_cmd_timed_launches.txt).
      hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
      if (r != hipSuccess) return (int32_t)r;
      marks.emplace_back(s, e);
      slot = &marks.back();
    }
    *out = slot->second;
    return (int32_t)hipEventRecord(slot->second, s);
  }
  void release() {
    for (auto& m : marks) {
      (void)hipEventSynchronize(m.second);
      (void)hipEventDestroy(m.second);
    }
    marks.clear();
  }
};

// The streams whose enqueued work reads or writes a buffer, each with the
// handle's event for that stream (StreamMarks, not owned here) recorded after
// that work.  The event may since have been recorded again, after later work:
// the tests below are conservative, never early.
struct StreamUses {
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
  // the calling stream has (just) enqueued work on the buffer; e: its mark
  void note(hipStream_t s, hipEvent_t e) {
    bool found = false;
    size_t j = 0;
    for (size_t i = 0; i < uses.size(); ++i) {
      if (uses[i].first == s) {
        uses[i].second = e;
        found = true;
      } else if (uses[i].second == e) {
        continue;  // the event moved to stream s: that stream's work completed
      }
      uses[j++] = uses[i];
    }
    uses.resize(j);
    if (!found) uses.emplace_back(s, e);
  }
  // every recorded use has completed (non-blocking)
  bool idle() const {
    for (const auto& u : uses)
      if (hipEventQuery(u.second) != hipSuccess) return false;
    return true;
  }
  // stream s waits (device side) for the uses on other streams
  int32_t order_after(hipStream_t s) const {
    for (const auto& u : uses)
      if (u.first != s) {
        hipError_t r = hipStreamWaitEvent(s, u.second, 0);
        if (r != hipSuccess) return (int32_t)r;
      }
    return 0;
  }
  void wait_all() const {
    for (const auto& u : uses) (void)hipEventSynchronize(u.second);
  }
  void release() { uses.clear(); }
};

// Compiled range tables (device) for one range set, with the key (packed
// bounds) they were compiled from and their pinned staging.  A handle keeps a
// few of them (LRU), so that alternating range sets -- the batched sums, the
// preview's single range, the multi-blob sensor's sticky range -- do not
// recompile, and a new range set never overwrites tables a queued kernel is
// still reading: it takes a set whose uses have all completed.
struct TableSet {
  std::vector<uint32_t> key;  // empty: unused
  int groups_cap = 0;
  RangeTables* d_tables = nullptr;
  RangeTables* h_tables = nullptr;
  StripeTables* d_stripe = nullptr;
  StripeTables* h_stripe = nullptr;
  ChromaTables* d_chroma = nullptr;        // built on first use per range set (chroma-run kernel)
  unsigned long long* h_cost = nullptr;    // pinned readback of each group's flagged_cost
  std::vector<uint8_t> detect;             // per group: detect_mode() of its ranges
  bool chroma_built = false;
  double chroma_share = -1.0;  // the builder's expected exact-path word share (max over groups), once read
  hipEvent_t ready = nullptr;       // uploads (and the chroma build) enqueued before it
  hipEvent_t cost_ready = nullptr;  // the flagged_cost readback enqueued before it
  StreamUses users;                 // kernels that read the set
  uint64_t tick = 0;                // last use (LRU)
  // AUTO's measured share per group: ChromaTables::flagged_words (the words
  // the chroma-run kernel's exact path resolved) read back every few
  // launches, over the words launched in between (Probe)
  struct Probe {
    uint64_t base = 0;          // the counter at the last landed readback
    bool have_base = false;
    uint64_t launched = 0;      // words launched on the chroma-run kernel since the last readback
    uint64_t in_flight = 0;     // those of the readback in flight
    // a gated launch (the device chose the kernel) since the last readback:
    // its words may or may not be in the counter, so that interval is not
    // measured (mixed) -- only the base moves
    bool mixed = false, in_flight_mixed = false;
    double measured = -1.0;     // flagged words / words between the last two readbacks
    int stripe_runs = 0;        // batches sent to the stripe kernel by the measured share
  };
  std::vector<Probe> probes;
  unsigned long long* h_words = nullptr;  // pinned [groups_cap]: the readback
  hipEvent_t words_ready = nullptr;
  bool words_pending = false;
  int chroma_runs = 0;  // calls with a chroma-run launch since the last readback
  void release() {
    users.wait_all();
    if (ready) (void)hipEventSynchronize(ready);
    if (words_ready) (void)hipEventSynchronize(words_ready);
    users.release();
    (void)hipFree(d_chroma);
    (void)hipHostFree(h_words);
    if (words_ready) (void)hipEventDestroy(words_ready);
    (void)hipHostFree(h_cost);
    (void)hipFree(d_tables);
    (void)hipHostFree(h_tables);
    (void)hipFree(d_stripe);
    (void)hipHostFree(h_stripe);
    if (ready) (void)hipEventDestroy(ready);
    if (cost_ready) (void)hipEventDestroy(cost_ready);
    *this = TableSet();
  }
  bool idle() const { return users.idle() && (!ready || hipEventQuery(ready) == hipSuccess); }
  // the exact-path share, once the readback has landed (-1 before)
  double share() {
    if (chroma_share < 0 && chroma_built && hipEventQuery(cost_ready) == hipSuccess) {
      double sh = 0.0;
      for (int g = 0; g < groups_cap; ++g) {
        const double v = (double)h_cost[g] / 4294967296.0;
        if (v > sh) sh = v;
      }
      chroma_share = sh;
    }
    return chroma_share;
  }
  // group g's own expected share (AUTO plans each group by its own tables),
  // or -1 while the builder's readback is in flight
  double group_share(int g) {
    if (!chroma_built || share() < 0) return -1.0;
    return (double)h_cost[g] / 4294967296.0;
  }
};
constexpr int kTableSets = 4;

struct TrikCvHandle {
  // XDAIS IALG_Obj: the framework's function table (algInit keeps it)
  TRIK_IALG_Obj ialg{};
  // false when the object lives in a framework-allocated IALG record
  // (algAlloc / algInit / algFree), true for TRIK_VIDTRANSCODE_CV_create
  bool owns_memory = true;
  int device = 0;
  int algo = kAlgoBall;
  // line sensor: the cross-point rows the previous run left (LSEQ:298 reads
  // m_hStart/m_hStop before LSEQ:449-450 sets them); set to the steady state
  // H/2, H/2+80 by setup (the reference leaves them uninitialised)
  int32_t line_band[2] = {0, 0};
  TRIK_VIDTRANSCODE_CV_Params params{};
  TRIK_VIDTRANSCODE_CV_DynamicParams dyn{};
  bool alg_ready = false;  // the reference's m_cvAlgorithm is set (WGLUE:302)
  int layout = TRIK_HSV_LAYOUT_YUYV;
  int in_w = 0, in_h = 0, in_ll = 0;
  int out_w = 0, out_h = 0, out_ll = 0;
  std::mutex mu;

  // compiled range tables (device), LRU over the range sets in use
  TableSet sets[kTableSets];
  uint64_t tick = 0;
  TableSet* sums_set = nullptr;  // the set of the last batched-sums call (trik_hsv_chroma_share)
  // hot-kernel choice for this handle (trik_hsv_set_hot_kernel) and the
  // kernel each range group of its last hot call ran (negative: the device
  // chose between the chroma-run kernel and -kind by the group's cost, the
  // share not being known yet; pending_set holds the costs), resolved by
  // trik_hsv_last_hot_kernel
  std::atomic<int> hot{TRIK_HSV_HOT_AUTO};
  std::atomic<int> reserved_cus{0};  // trik_hsv_set_reserved_cus
  std::vector<int8_t> hot_groups;
  TableSet* pending_set = nullptr;

  // preview geometry: scale maps for maps_key = {W, H, out_w, out_h}
  uint32_t* d_maps = nullptr;
  size_t d_maps_cap = 0;
  int maps_key[6] = {-1, -1, -1, -1, -1, -1};
  int32_t maps_rows2 = -1;  // first source row when the maps are the 2:1 ones, else -1
  int32_t maps_guides = 0;  // the guide lines' output bits follow the maps (2:1 maps)
  int32_t maps_rows2_c0 = 0, maps_rows2_c1 = 0;  // the output columns the 2:1 maps write
  // the line sensors' overlay geometry on these maps (PreviewArgs::ovl_*)
  int32_t maps_ovl_half = 0, maps_ovl_ok = 0, maps_ovl_mag[4] = {-1, -1, -1, -1}, maps_ovl_band[2] = {-1, -1};
  int32_t maps_ovl_c_lo = 0, maps_ovl_c_hi = -1;
  std::vector<uint32_t> h_maps;
  StreamUses maps_users;

  // process() staging
  hipStream_t stream = nullptr;
  uint8_t* d_preview = nullptr;
  size_t d_preview_cap = 0;
  uint16_t* d_auto = nullptr;
  uint8_t* d_frame = nullptr;
  size_t d_frame_cap = 0;
  TrikHsvTargetSums* d_sums = nullptr;
  TrikHsvTarget* d_targets = nullptr;

  // the chroma-run kernel's fused step: per-workgroup partial totals and the
  // last-workgroup counter, per-frame accumulators and unit-done counts (all
  // zero between launches), shared by this handle's calls
  unsigned long long* d_wg_part = nullptr;
  uint32_t* d_wg_cnt = nullptr;
  unsigned long long* d_frame_acc = nullptr;  // [frames][16]: 12 sums, the unit count
  int64_t frame_acc_cap = 0;  // frames
  StreamUses fused_users;
  // the chroma-run kernel's sink for its past-the-end loads (KernelArgs::tail):
  // kChromaTailSink bytes, allocated once on first use, never resized
  uint8_t* d_tail_sink = nullptr;

  // ov7670 multi-blob sensor: BitmapBuilder's sticky range (uninitialised in
  // the reference before the first setHsvRange; zero here) and scratch
  TRIK_VIDTRANSCODE_CV_InArgsAlg blob_range{};  // as webcam-form bounds (all zero at first)
  uint8_t* d_meta = nullptr;
  size_t d_meta_cap = 0;
  int32_t* d_blob_stats = nullptr;
  size_t d_blob_stats_cap = 0;
  bool blob_stats_dirty = false;  // zeroed whole by the next call (a failed clusterer launch)
  int32_t* d_blob_top = nullptr;
  size_t d_blob_top_cap = 0;
  TrikHsvTarget* d_blob_targets = nullptr;
  size_t d_blob_targets_cap = 0;
  StreamUses blob_users;  // calls that wrote the multi-blob scratch
  StreamMarks marks;      // the events the StreamUses lists point at (freed last)
};

namespace {

// The handle's device resources, freed; the object stays valid (null
// pointers, no streams), so that this may run twice.
void free_resources(TrikCvHandle* h) {
  int prev = 0;
  bool switched = hipGetDevice(&prev) == hipSuccess && prev != h->device &&
                  hipSetDevice(h->device) == hipSuccess;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (TableSet& t : h->sets) t.release();
  h->maps_users.wait_all();
  h->maps_users.release();
  h->blob_users.wait_all();
  h->blob_users.release();
  h->fused_users.wait_all();
  h->fused_users.release();
  h->marks.release();
  (void)hipFree(h->d_wg_part);
  (void)hipFree(h->d_frame_acc);
  (void)hipFree(h->d_tail_sink);
  (void)hipFree(h->d_frame);
  (void)hipFree(h->d_maps);
  (void)hipFree(h->d_preview);
  (void)hipFree(h->d_auto);
  (void)hipFree(h->d_sums);
  (void)hipFree(h->d_targets);
  (void)hipFree(h->d_meta);
  (void)hipFree(h->d_blob_stats);
  (void)hipFree(h->d_blob_top);
  (void)hipFree(h->d_blob_targets);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  if (switched) (void)hipSetDevice(prev);
  h->stream = nullptr;
  h->d_frame = nullptr; h->d_frame_cap = 0;
  h->d_maps = nullptr; h->d_maps_cap = 0;
  h->maps_key[0] = -1;
  h->d_preview = nullptr; h->d_preview_cap = 0;
  h->d_auto = nullptr;
  h->d_sums = nullptr;
  h->d_targets = nullptr;
  h->d_meta = nullptr; h->d_meta_cap = 0;
  h->d_blob_stats = nullptr; h->d_blob_stats_cap = 0;
  h->d_blob_top = nullptr; h->d_blob_top_cap = 0;
  h->d_blob_targets = nullptr; h->d_blob_targets_cap = 0;
  h->d_wg_part = nullptr; h->d_wg_cnt = nullptr;
  h->d_frame_acc = nullptr; h->frame_acc_cap = 0;
  h->d_tail_sink = nullptr;
  h->sums_set = h->pending_set = nullptr;
  h->alg_ready = false;
}

void release(TrikCvHandle* h) {
  if (!h) return;
  free_resources(h);
  if (h->owns_memory)
    delete h;
  else
    h->~TrikCvHandle();  // the framework releases the record (algFree)
}

// handleSetupImageDesc + createCVAlgorithm + BallDetector::setup
// (WGLUE:52-145, WSEQ:358-410).
int32_t setup_image_desc(TrikCvHandle* h) {
  h->alg_ready = false;
  const TRIK_IVIDTRANSCODE_Params& p = h->params.base;
  if (p.numOutputStreams != 0 && p.numOutputStreams != 1)  // WGLUE:96-101
    return fail(TRIK_IALG_EFAIL, "invalid number of output streams");
  const int in_fmt = p.formatInput;
  const int in_w = h->dyn.inputWidth > 0 ? h->dyn.inputWidth : 0;  // WGLUE:106-109
  const int in_h = h->dyn.inputHeight > 0 ? h->dyn.inputHeight : 0;
  const int in_ll = h->dyn.inputLineLength > 0 ? h->dyn.inputLineLength : 0;
  int out_fmt = TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_UNKNOWN, out_w = 0, out_h = 0, out_ll = 0;
  if (p.numOutputStreams == 1) {  // WGLUE:111-117
    out_fmt = p.formatOutput[0];
    out_w = h->dyn.base.outputWidth[0] > 0 ? h->dyn.base.outputWidth[0] : 0;
    out_h = h->dyn.base.outputHeight[0] > 0 ? h->dyn.base.outputHeight[0] : 0;
    out_ll = h->dyn.outputLineLength[0] > 0 ? h->dyn.outputLineLength[0] : 0;
  }
  if (in_w > p.maxWidthInput || in_h > p.maxHeightInput ||  // WGLUE:126-135
      (p.numOutputStreams == 1 && (out_w > p.maxWidthOutput[0] || out_h > p.maxHeightOutput[0])))
    return fail(TRIK_IALG_EFAIL, "invalid image dimensions");
  // IF_IN_OUT_FORMAT dispatch (WGLUE:76-84): BallDetector<YUV422, RGB565X>
  // (webcam) and BallDetector<YUV422P, RGB565X> (ov7670 object sensor).  With
  // no output stream the preview format is UNKNOWN; the reference then finds
  // no algorithm, this build accepts it (no preview to write).
  const bool out_ok = out_fmt == TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_RGB565X ||
                      (p.numOutputStreams == 0 && out_fmt == TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_UNKNOWN);
  int layout;
  if (h->algo == kAlgoBlob &&
      (in_w > 8192 || blob_max_labels(in_w / 4, in_h / 4) > 30000))  // uint16 labels, LDS
    return fail(TRIK_IALG_EFAIL, "CV algorithm setup failed: frame too large for the multi-blob sensor");
  if ((h->algo == kAlgoBall || h->algo == kAlgoWLine) && in_fmt == TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422 &&
      out_ok)
    layout = TRIK_HSV_LAYOUT_YUYV;
  else if (h->algo != kAlgoWLine && in_fmt == TRIK_VIDTRANSCODE_CV_VIDEO_FORMAT_YUV422P &&
           out_ok)  // ov7670 line: YUV422P only; webcam line: YUV422 only
    layout = TRIK_HSV_LAYOUT_OV7670;
  else
    return fail(TRIK_IALG_EFAIL, "cannot create CV algorithm for this format pair");
  if (in_w % 32 != 0 || in_h % 4 != 0 || in_w > 32767 || in_h > 32767)  // WSEQ:365-369
    return fail(TRIK_IALG_EFAIL, "CV algorithm setup failed: width % 32 / height % 4");
  const int row = layout == TRIK_HSV_LAYOUT_YUYV ? 2 * in_w : in_w;
  if (in_h > 0 && in_ll < row)
    return fail(TRIK_IALG_EFAIL, "CV algorithm setup failed: inputLineLength shorter than a row");
  h->layout = layout;
  h->in_w = in_w; h->in_h = in_h; h->in_ll = in_ll;
  h->out_w = out_w; h->out_h = out_h; h->out_ll = out_ll;
  h->line_band[0] = in_h / 2;
  h->line_band[1] = in_h / 2 + 80;
  h->alg_ready = true;
  return TRIK_IALG_EOK;
}

int32_t setup_dynamic(TrikCvHandle* h, const TRIK_VIDTRANSCODE_CV_DynamicParams* d) {
  h->dyn = d ? *d : default_dynamic_params(h->algo);  // WGLUE:271-274
  return setup_image_desc(h);
}

// The last call's gated groups (hot_groups[g] = -partner: AUTO's choice made
// on the device from the builder cost) resolved from that cost, which was
// copied back without a host wait: waits for the copy.  Runs when the answer
// is asked for and before the pending set's slot is reused.
void resolve_pending(TrikCvHandle* h) {
  TableSet* t = h->pending_set;
  if (!t) return;
  (void)hipEventSynchronize(t->cost_ready);
  for (size_t g = 0; g < h->hot_groups.size(); ++g)
    if (h->hot_groups[g] < 0)
      h->hot_groups[g] = (int8_t)(g < (size_t)t->groups_cap && t->h_cost[g] <= kChromaMaxCost ? TRIK_HSV_HOT_CHROMA
                                                                                             : -h->hot_groups[g]);
  h->pending_set = nullptr;
}

// The tables for ranges[0..n), stream-ordered on s: a cached set (s waits
// for its uploads, device side), or a set compiled now into a slot whose
// earlier uses have completed -- found without blocking (hipEventQuery);
// only when all kTableSets sets are still in use does the host wait for the
// least recently used one.
int32_t acquire_tables(TrikCvHandle* h, const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, hipStream_t s,
                       TableSet** out) {
  std::vector<uint32_t> key;
  key.reserve(3 * n + 1);
  key.push_back((uint32_t)n);
  for (int i = 0; i < n; ++i) {
    const PackedRange p = pack_range(ranges[i]);
    key.push_back(p.from); key.push_back(p.to); key.push_back(p.expect);
  }
  for (TableSet& t : h->sets)
    if (!t.key.empty() && t.key == key) {
      if (t.ready) HIP_TRY(hipStreamWaitEvent(s, t.ready, 0));
      t.tick = ++h->tick;
      *out = &t;
      return 0;
    }
  TableSet* v = nullptr;
  for (TableSet& t : h->sets)
    if (t.key.empty()) { v = &t; break; }
  if (!v)
    for (TableSet& t : h->sets)
      if (t.idle() && (!v || t.tick < v->tick)) v = &t;
  if (!v) {  // every set is in use: wait for the least recently used one
    for (TableSet& t : h->sets)
      if (!v || t.tick < v->tick) v = &t;
    v->users.wait_all();
    if (v->ready) HIP_TRY(hipEventSynchronize(v->ready));
  }
  if (h->pending_set == v) resolve_pending(h);  // (its costs are about to be overwritten)
  if (h->sums_set == v) h->sums_set = nullptr;
  const int groups = (n + kRangesPerLaunch - 1) / kRangesPerLaunch;
  if (groups > v->groups_cap) {
    v->release();
    HIP_TRY(hipMalloc(&v->d_tables, sizeof(RangeTables) * groups));
    HIP_TRY(hipHostMalloc(&v->h_tables, sizeof(RangeTables) * groups, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&v->d_stripe, sizeof(StripeTables) * groups));
    HIP_TRY(hipHostMalloc(&v->h_stripe, sizeof(StripeTables) * groups, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&v->h_cost, sizeof(unsigned long long) * groups, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc(&v->h_words, sizeof(unsigned long long) * groups, hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&v->words_ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&v->ready, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&v->cost_ready, hipEventDisableTiming));
    v->groups_cap = groups;
  }
  v->key.clear();  // invalid until the uploads are enqueued
  // the set's earlier uploads and readers have finished (idle), so its pinned
  // staging and device tables may be rewritten
  v->detect.assign(groups, kDetectFull);
  // the tables: built on the device from the packed ranges (no table crosses
  // PCIe: a host-built upload went through the copy engine, whose hand-offs
  // with the compute queue cost tens of microseconds); the per-value tests
  // are also compiled on the host, for detect_mode
  TableBuildArgs ta = {};
  ta.n_ranges = n;
  for (int i = 0; i < n && groups <= kTableGroups; ++i) {
    const PackedRange p = pack_range(ranges[i]);
    ta.from[i] = p.from;
    ta.to[i] = p.to;
    ta.expect[i] = p.expect;
  }
  for (int g = 0; g < groups; ++g) {
    const int cnt = n - g * kRangesPerLaunch < kRangesPerLaunch ? n - g * kRangesPerLaunch : kRangesPerLaunch;
    if (groups <= kTableGroups) {
      compile_tables_head(ranges + g * kRangesPerLaunch, cnt, &v->h_tables[g]);
    } else {  // (more than 64 ranges: compiled on the host, uploaded below)
      compile_tables(ranges + g * kRangesPerLaunch, cnt, &v->h_tables[g]);
      compile_stripe_tables(v->h_tables[g], cnt, &v->h_stripe[g]);
    }
    v->detect[g] = (uint8_t)detect_mode(v->h_tables[g], cnt);
  }
  if (groups == 0) {
  } else if (groups <= kTableGroups) {
    HIP_TRY(launch_compile_tables(ta, groups, v->d_tables, v->d_stripe, s));
  } else {
    HIP_TRY(hipMemcpyAsync(v->d_tables, v->h_tables, sizeof(RangeTables) * groups, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(v->d_stripe, v->h_stripe, sizeof(StripeTables) * groups, hipMemcpyHostToDevice, s));
  }
  HIP_TRY(hipEventRecord(v->ready, s));
  v->key.swap(key);
  v->chroma_built = false;
  v->chroma_share = -1.0;
  if (v->words_pending) (void)hipEventSynchronize(v->words_ready);
  v->words_pending = false;
  v->probes.assign(groups, TableSet::Probe());
  v->chroma_runs = 0;
  v->tick = ++h->tick;
  *out = v;
  return 0;
}

// The chroma-run kernel's tables for the set's range groups, built on the
// device from the uploaded RangeTables (stream-ordered on s).  The builder's
// expected exact-path cost is copied back into pinned memory without waiting:
// TableSet::share() reads it once it has landed.
int32_t ensure_chroma(TableSet& t, int groups, hipStream_t s) {
  if (t.chroma_built) return 0;
  if (!t.d_chroma) HIP_TRY(hipMalloc(&t.d_chroma, sizeof(ChromaTables) * t.groups_cap));
  for (int g = 0; g < groups; ++g) {
    HIP_TRY(build_chroma_tables(t.d_tables + g, t.d_chroma + g, s));
    HIP_TRY(hipMemcpyAsync(&t.h_cost[g], &t.d_chroma[g].flagged_cost, sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, s));
  }
  for (int g = groups; g < t.groups_cap; ++g) t.h_cost[g] = 0;
  HIP_TRY(hipEventRecord(t.cost_ready, s));
  HIP_TRY(hipEventRecord(t.ready, s));  // later users on other streams wait for the build too
  t.chroma_built = true;
  t.chroma_share = -1.0;
  return 0;
}

// How the hot kernel is chosen for one launch: CHROMA / STRIPE decided on the
// host, or GATED: both launched, the device picks by the builder's cost.
enum HotPlan { kPlanStripe, kPlanChroma, kPlanGated };

// Batches AUTO keeps on the stripe kernel for a group whose measured share
// is too high before it tries the chroma-run kernel again (re-measuring), and
// AUTO chroma-run launches between readbacks of the measured share.
constexpr int kReprobeAfter = 32;
constexpr int kProbeEvery = 8;

// The measured shares, once their readback has landed (non-blocking).
void poll_measured(TableSet& t) {
  if (!t.words_pending || hipEventQuery(t.words_ready) != hipSuccess) return;
  for (size_t g = 0; g < t.probes.size(); ++g) {
    TableSet::Probe& p = t.probes[g];
    const uint64_t v = t.h_words[g];
    if (p.have_base && p.in_flight > 0 && !p.in_flight_mixed)
      p.measured = (double)(v - p.base) / (double)p.in_flight;
    p.base = v;
    p.have_base = true;
    p.in_flight = 0;
    p.in_flight_mixed = false;
  }
  t.words_pending = false;
}

HotPlan plan_hot(TrikCvHandle* h, TableSet& t, int g, int groups, bool big, bool chroma_ok, hipStream_t s,
                 int32_t* rc) {
  *rc = 0;
  const int choice = h->hot.load();
  if (!chroma_ok || !(choice == TRIK_HSV_HOT_CHROMA || (choice == TRIK_HSV_HOT_AUTO && big))) return kPlanStripe;
  *rc = ensure_chroma(t, groups, s);
  if (*rc) return kPlanStripe;
  if (choice == TRIK_HSV_HOT_CHROMA) return kPlanChroma;
  const double sh = t.group_share(g);
  if (sh < 0) return kPlanGated;  // the share is still in flight: no host wait
  if (sh > TRIK_HSV_CHROMA_MAX_SHARE) return kPlanStripe;
  // the input's own share, measured on earlier batches: input that
  // concentrates on the chromas the tables describe worst (their windows and
  // exceptions) goes to the stripe kernel, with a chroma-run batch now and
  // then to see whether it still does
  TableSet::Probe& p = t.probes[g];
  if (p.measured > TRIK_HSV_CHROMA_MAX_SHARE && ++p.stripe_runs <= kReprobeAfter) return kPlanStripe;
  p.stripe_runs = 0;
  return kPlanChroma;
}

// After a call's launches: AUTO chroma-run words counted, and every
// kProbeEvery such launches (or right after a re-probe) the groups' exact-path
// word counters read back into pinned memory without a host wait.
int32_t probe_measured(TableSet& t, bool reprobe, hipStream_t s) {
  if (t.chroma_runs == 0 || t.words_pending) return 0;
  bool want = reprobe || t.chroma_runs >= kProbeEvery;
  for (const TableSet::Probe& p : t.probes) want = want || !p.have_base;
  if (!want) return 0;
  const size_t n = t.probes.size();
  for (size_t g = 0; g < n; ++g)
    HIP_TRY(hipMemcpyAsync(&t.h_words[g], &t.d_chroma[g].flagged_words, sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, s));
  HIP_TRY(hipEventRecord(t.words_ready, s));
  for (TableSet::Probe& p : t.probes) {
    p.in_flight = p.launched;
    p.in_flight_mixed = p.mixed;
    p.launched = 0;
    p.mixed = false;
  }
  t.words_pending = true;
  t.chroma_runs = 0;
  return 0;
}

// The outputs of a full step (process_batch): sums written whole (not added),
// targets and the per-target batch totals when not NULL.
struct StepOut {
  TrikHsvTarget* targets = nullptr;
  TrikHsvTargetSums* totals = nullptr;
};

// Record that the work just enqueued on s reads `set` (and the preview maps,
// and `extra`): one event record on s for the call.
int32_t note_uses(TrikCvHandle* h, TableSet* set, bool maps, hipStream_t s, StreamUses* extra = nullptr) {
  hipEvent_t e = nullptr;
  int32_t r = h->marks.mark(s, &e);
  if (r) return fail(TRIK_IVIDTRANSCODE_EFAIL, std::string("hipEventRecord: ") + hipGetErrorString((hipError_t)r));
  if (set) set->users.note(s, e);
  if (maps) h->maps_users.note(s, e);
  if (extra) extra->note(s, e);
  return 0;
}

// The fused step's scratch, allocated on first use: one slot of 12 totals per
// CU and the last-workgroup counter; per frame a 128-byte line holding its 12
// accumulators and its unit-done count.  All zeroed once; every launch leaves
// them zero.  A larger batch reallocates the per-frame part (after the
// launches still using it: the caller ordered s after them).
int32_t ensure_fused_scratch(TrikCvHandle* h, int64_t n_frames, hipStream_t s) {
  if (!h->d_wg_part) {
    const size_t parts = (size_t)device_cus() * 12;
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, sizeof(unsigned long long) * parts + 16));
    h->d_wg_part = static_cast<unsigned long long*>(p);
    h->d_wg_cnt = reinterpret_cast<uint32_t*>(h->d_wg_part + parts);
    HIP_TRY(hipMemsetAsync(h->d_wg_cnt, 0, 16, s));
  }
  if (n_frames > h->frame_acc_cap) {
    if (h->d_frame_acc) {
      HIP_TRY(hipStreamSynchronize(s));
      (void)hipFree(h->d_frame_acc);
      h->d_frame_acc = nullptr;
      h->frame_acc_cap = 0;
    }
    const int64_t cap = n_frames < 1024 ? 1024 : n_frames;
    const size_t bytes = (size_t)cap * 128;
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes));
    HIP_TRY(hipMemsetAsync(p, 0, bytes, s));
    h->d_frame_acc = static_cast<unsigned long long*>(p);
    h->frame_acc_cap = cap;
  }
  return 0;
}

// The hot kernel(s) over the batch: one launch per group of <= 4 ranges.
// Without `step` the kernels ADD into sums (the caller zeroes it).  With it
// the call is a full step: when every group runs the chroma-run kernel and the
// batch gives each workgroup whole frames (chroma_fused_ok), each launch
// zeroes its sums and writes its targets and totals itself (the fused step,
// one launch per group); otherwise sums are zeroed first and the epilogue and
// totals kernels follow.
int32_t run_sums(TrikCvHandle* h, const TrikHsvFrameBatch* b,
                 const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int n, TrikHsvTargetSums* sums,
                 uint8_t* masks, hipStream_t s, const StepOut* step = nullptr) {
  TableSet* t = nullptr;
  int32_t rc = acquire_tables(h, ranges, n, s, &t);
  if (rc) return rc;
  h->sums_set = t;
  const bool empty = b->n_frames == 0 || b->width == 0 || b->height == 0;
  const int groups = (n + kRangesPerLaunch - 1) / kRangesPerLaunch;
  const bool big = (int64_t)b->n_frames * b->width * b->height >= (int64_t)TRIK_HSV_CHROMA_MIN_PIXELS;
  std::vector<KernelArgs> args(empty ? 0 : groups);
  std::vector<HotPlan> plans(args.size(), kPlanStripe);
  bool fused = step != nullptr && !masks && !empty;
  poll_measured(*t);
  bool reprobe = false;
  for (size_t g = 0; g < args.size(); ++g) {
    KernelArgs& a = args[g];
    a.frames = static_cast<const uint8_t*>(b->frames);
    a.frame_stride = b->n_frames > 1 ? b->frame_stride : 0;
    a.n_frames = b->n_frames;
    a.width = b->width; a.height = b->height; a.line_length = b->line_length;
    a.layout = b->layout;
    a.n_ranges = n - (int)g * kRangesPerLaunch < kRangesPerLaunch ? n - (int)g * kRangesPerLaunch : kRangesPerLaunch;
    a.range_offset = (int)g * kRangesPerLaunch;
    a.sums_ranges = n;
    a.tables = t->d_tables + g;
    a.stripe_tables = t->d_stripe + g;
    a.detect_mode = t->detect[g];
    a.sums = sums;
    a.masks = masks;
    a.mask_shift = (int)g * kRangesPerLaunch;
    // the chroma-run kernel for large batches, the stripe kernel otherwise;
    // the generic kernel takes misaligned inputs and rows wider than 8192 pixels
    // value-only groups (every range accepts every hue and saturation) run
    // the stripe kernel's value form under AUTO at any batch size: it beats
    // the chroma-run kernel there and needs no table build
    const bool was_measured_stripe = g < t->probes.size() && t->probes[g].stripe_runs > 0;
    plans[g] = plan_hot(h, *t, (int)g, groups, big && t->detect[g] != kDetectV,
                        h->hot.load() != TRIK_HSV_HOT_GENERIC && chroma_geometry_ok(a), s, &rc);
    if (rc) return rc;
    reprobe = reprobe || (was_measured_stripe && plans[g] == kPlanChroma);
    fused = fused && plans[g] == kPlanChroma && chroma_fused_ok(a);
  }
  if (fused) {
    HIP_TRY(h->fused_users.order_after(s));
    rc = ensure_fused_scratch(h, b->n_frames, s);
    if (rc) return rc;
  }
  bool any_chroma = false;
  for (HotPlan p : plans) any_chroma = any_chroma || p != kPlanStripe;
  if (any_chroma && !h->d_tail_sink) {  // (its contents are never used: zeroed once for tidiness)
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, (size_t)kChromaTailSink));
    HIP_TRY(hipMemsetAsync(p, 0, (size_t)kChromaTailSink, s));
    h->d_tail_sink = static_cast<uint8_t*>(p);
  }
  for (KernelArgs& a : args) {
    a.tail = h->d_tail_sink;
    a.tail_bytes = h->d_tail_sink ? kChromaTailSink : 0;
    a.reserved_cus = h->reserved_cus.load();
  }
  if (step && !fused && b->n_frames > 0 && sums)  // (frames of zero width or height: zero sums)
    HIP_TRY(hipMemsetAsync(sums, 0, sizeof(TrikHsvTargetSums) * (size_t)b->n_frames * n, s));
  bool gated = false, chroma_ran = false;
  // (an empty batch launches nothing and keeps the last call's answer)
  if (!args.empty()) {
    h->hot_groups.assign(groups, 0);
    h->pending_set = nullptr;  // (set again as soon as a group is gated)
  }
  for (size_t g = 0; g < args.size(); ++g) {
    KernelArgs& a = args[g];
    const HotPlan plan = plans[g];
    int e = hipErrorNotSupported;
    if (plan == kPlanChroma) {
      if (fused) {
        a.fused = 1;
        a.targets = step->targets;
        a.totals = step->totals;
        a.wg_part = h->d_wg_part;
        a.wg_cnt = h->d_wg_cnt;
        a.frame_acc = h->d_frame_acc;
      }
      e = launch_chroma(a, t->d_chroma + g, masks != nullptr, s);
      if (e == hipSuccess) {
        h->hot_groups[g] = TRIK_HSV_HOT_CHROMA;
        // every chroma-run launch adds to the group's flagged_words (forced or
        // AUTO), so every one counts its words: the two sides of the share
        t->probes[g].launched += (uint64_t)a.n_frames * (uint64_t)(a.width / 2) * (uint64_t)a.height;
        chroma_ran = true;
      }
    } else if (plan == kPlanGated) {
      // AUTO's rule on the device: the chroma-run kernel runs while this
      // group's cost is at most kChromaMaxCost, its partner otherwise -- the
      // stripe kernel, or the generic kernel where the stripe kernel's
      // geometry does not take the batch (rows wider than 8192 pixels), with
      // the same gate: exactly one of the two adds into the sums
      KernelArgs ac = a, as = a;
      ac.gate = as.gate = &t->d_chroma[g].flagged_cost;
      ac.gate_max = as.gate_max = kChromaMaxCost;
      ac.gate_le = 1;
      as.gate_le = 0;
      e = launch_chroma(ac, t->d_chroma + g, masks != nullptr, s);
      if (e == hipSuccess) {
        int partner = TRIK_HSV_HOT_STRIPE;
        e = launch_stripe(as, masks != nullptr, s);
        if (e == hipErrorNotSupported) {
          partner = TRIK_HSV_HOT_GENERIC;
          e = launch_reduce(as, masks != nullptr, s);
        }
        HIP_TRY(e);  // never an ungated launch after a gated one
        h->hot_groups[g] = (int8_t)-partner;
        h->pending_set = t;  // at once: a later group's error return leaves it consistent
        t->probes[g].mixed = true;
        gated = true;
        continue;
      }
    }
    if (e == hipErrorNotSupported && h->hot.load() != TRIK_HSV_HOT_GENERIC) {
      e = launch_stripe(a, masks != nullptr, s);
      if (e == hipSuccess) h->hot_groups[g] = TRIK_HSV_HOT_STRIPE;
    }
    if (e == hipErrorNotSupported) {
      e = launch_reduce(a, masks != nullptr, s);
      if (e == hipSuccess) h->hot_groups[g] = TRIK_HSV_HOT_GENERIC;
    }
    HIP_TRY(e);
  }
  // (an empty batch keeps the last call's answer, gated groups included)
  if (!args.empty()) h->pending_set = gated ? t : nullptr;
  if (chroma_ran) ++t->chroma_runs;  // once per call, whichever groups ran it
  if (!masks) {
    rc = probe_measured(*t, reprobe, s);
    if (rc) return rc;
  }
  if (step && !fused) {  // the epilogue and the totals as kernels of their own
    if (step->targets) HIP_TRY(launch_targets(*b, n, sums, step->targets, s));
    if (step->totals) HIP_TRY(launch_totals(b->n_frames > 0 ? b->n_frames : 0, n, sums, step->totals, s));
  }
  return note_uses(h, t, false, s, fused ? &h->fused_users : nullptr);
}

inline void set_bit(int32_t& word, int bit) { word |= (int32_t)(1u << bit); }

// Scale maps of the preview (WSEQ:371-387) for this geometry, uploaded once.
// col_lo..col_hi: the source columns that write (the line sensor's window).
// A geometry change (rare) waits for the kernels still reading the old maps
// and for the upload (the staging is pageable and reused).
int32_t ensure_maps(TrikCvHandle* h, int w, int hgt, int ow, int oh, hipStream_t s, int col_lo = 0,
                    int col_hi = 0x7FFFFFFF) {
  if (h->d_maps && h->maps_key[0] == w && h->maps_key[1] == hgt && h->maps_key[2] == ow &&
      h->maps_key[3] == oh && h->maps_key[4] == col_lo && h->maps_key[5] == col_hi)
    return 0;
  const size_t n = (size_t)w + hgt + ow + oh;
  h->maps_users.wait_all();  // previous users done
  h->h_maps.assign(n ? n : 1, 0u);
  preview_maps(w, hgt, ow, oh, h->h_maps.data(), col_lo, col_hi);
  // the 2:1 maps (the defaults' 640x480 -> 320x240): preview_rows2_kernel
  bool rows2 = false;
  int c0 = 0, c1 = ow;
  {
    const uint32_t* last_row = h->h_maps.data() + w + hgt;
    const uint32_t* last_col = last_row + oh;
    rows2 = oh > 0 && ow > 0 && (int32_t)last_row[0] >= 0;
    for (int r = 0; rows2 && r < oh; ++r) rows2 = (int32_t)last_row[r] == (int32_t)last_row[0] + 2 * r;
    // the written columns: one window [c0, c1) with last_col[c] = 2c + 1, -1 outside
    while (c0 < ow && (int32_t)last_col[c0] < 0) ++c0;
    while (c1 > c0 && (int32_t)last_col[c1 - 1] < 0) --c1;
    for (int c = 0; rows2 && c < ow; ++c)
      rows2 = (c >= c0 && c < c1) ? (int32_t)last_col[c] == 2 * c + 1 : (int32_t)last_col[c] < 0;
    h->maps_rows2 = rows2 ? (int32_t)last_row[0] : -1;
  }
  h->maps_rows2_c0 = c0;
  h->maps_rows2_c1 = c1;
  // The object sensors' 8 guide lines (draw_guides, WSEQ:136-166,471-485) as
  // output pixels, one bit each, 8 per byte along a row, behind the maps: the
  // 2:1 row kernel writes them as it writes the preview, so the overlay only
  // draws the target circle.  The same points and clamping as Canvas::px.
  h->maps_guides = 0;
  if (rows2 && ow % 8 == 0 && w > 0 && hgt > 0) {
    const size_t gpr = (size_t)ow / 8, words = ((size_t)oh * gpr + 3) / 4;
    h->h_maps.resize(n + words, 0u);
    uint8_t* bits = reinterpret_cast<uint8_t*>(h->h_maps.data() + n);
    const uint32_t* wi2wo = h->h_maps.data();
    const uint32_t* hi2ho = wi2wo + w;
    const auto px = [&](int col, int row) {
      const int sc = col < 0 ? 0 : (col > w - 1 ? w - 1 : col);
      const int sr = row < 0 ? 0 : (row > hgt - 1 ? hgt - 1 : row);
      const uint32_t oc = wi2wo[sc], orow = hi2ho[sr];
      if (oc < (uint32_t)ow && orow < (uint32_t)oh) bits[orow * gpr + oc / 8] |= (uint8_t)(1u << (oc % 8));
    };
    const int step = hgt / 6, hh = hgt / 2, hw = w / 2;
    for (int k = 0; k < 8 * 100; ++k) {
      const int line = k / 100, adj = k % 100, off = (line & 3) < 2 ? ((line & 3) - 2) : ((line & 3) - 1);
      if (line < 4) {
        px(hw + off * step, hh - adj);
        px(hw + off * step, hh + adj);
      } else {
        px(hw - adj, hh + off * step);
        px(hw + adj, hh + off * step);
      }
    }
    h->maps_guides = 1;
  }
  const size_t total = h->h_maps.size();
  if (total > h->d_maps_cap) {
    (void)hipFree(h->d_maps);
    h->d_maps = nullptr; h->d_maps_cap = 0;
    HIP_TRY(hipMalloc(&h->d_maps, sizeof(uint32_t) * total));
    h->d_maps_cap = total;
  }
  HIP_TRY(hipMemcpyAsync(h->d_maps, h->h_maps.data(), sizeof(uint32_t) * total, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));  // h_maps is pageable and reused
  h->maps_key[0] = w; h->maps_key[1] = hgt; h->maps_key[2] = ow; h->maps_key[3] = oh;
  h->maps_key[4] = col_lo; h->maps_key[5] = col_hi;
  // the line overlays' output pixels (line_overlay_kernel, LSEQ:419-474): a
  // column map with steps of 0 or 1 sends any source interval to one interval
  const uint32_t* wi2wo = h->h_maps.data();
  const uint32_t* hi2ho = wi2wo + w;
  bool step1 = w > 0 && hgt > 0;
  for (int c = 1; step1 && c < w; ++c) step1 = wi2wo[c] - wi2wo[c - 1] <= 1u;
  h->maps_ovl_ok = step1 ? 1 : 0;
  bool half = step1;
  for (int c = 0; half && c < w; ++c) half = wi2wo[c] == (uint32_t)c >> 1;
  h->maps_ovl_half = half ? 1 : 0;
  if (step1) {
    const auto cl = [](int v, int n) { return v < 0 ? 0 : (v > n - 1 ? n - 1 : v); };
    const int hw = w / 2, hh = hgt / 2, step = 40;
    const int cols[4] = {hw - step, hw + step, hw - 2 * step, hw + 2 * step};
    for (int j = 0; j < 4; ++j) h->maps_ovl_mag[j] = (int32_t)wi2wo[cl(cols[j], w)];
    h->maps_ovl_band[0] = (int32_t)hi2ho[cl(hh, hgt)];
    h->maps_ovl_band[1] = (int32_t)hi2ho[cl(hh + 2 * step, hgt)];
    h->maps_ovl_c_lo = (int32_t)wi2wo[0];
    h->maps_ovl_c_hi = (int32_t)wi2wo[w - 1];
  }
  return 0;
}

PreviewArgs preview_args(const TrikCvHandle* h, const TrikHsvFrameBatch& b,
                         const TRIK_VIDTRANSCODE_CV_InArgsAlg& range, int ow, int oh, int oll,
                         uint8_t* previews, int64_t stride) {
  PreviewArgs a;
  a.frames = static_cast<const uint8_t*>(b.frames);
  a.frame_stride = b.frame_stride;
  a.n_frames = b.n_frames;
  a.width = b.width; a.height = b.height; a.line_length = b.line_length; a.layout = b.layout;
  a.range = pack_range(range);
  const auto al = [](int64_t v) { return (v & 3) == 0; };
  a.aligned4 = al((int64_t)reinterpret_cast<uintptr_t>(b.frames)) && (b.n_frames <= 1 || al(b.frame_stride)) &&
               al(b.line_length) && al((int64_t)reinterpret_cast<uintptr_t>(previews)) &&
               (b.n_frames <= 1 || al(stride)) && al(oll);
  a.out_w = ow; a.out_h = oh; a.out_ll = oll;
  a.previews = previews;
  a.preview_stride = stride;
  a.wi2wo = h->d_maps;
  a.hi2ho = a.wi2wo + b.width;
  a.last_row = reinterpret_cast<const int32_t*>(a.hi2ho + b.height);
  a.last_col = a.last_row + oh;
  a.rows2_first = h->maps_rows2;
  if (h->maps_guides) a.guide_bits = reinterpret_cast<const uint8_t*>(h->d_maps + b.width + b.height + ow + oh);
  a.rows2_c0 = h->maps_rows2_c0;
  a.rows2_c1 = h->maps_rows2_c1;
  a.ovl_ok = h->maps_ovl_ok;
  a.ovl_half = h->maps_ovl_half;
  for (int j = 0; j < 4; ++j) a.ovl_mag[j] = h->maps_ovl_mag[j];
  a.ovl_band[0] = h->maps_ovl_band[0];
  a.ovl_band[1] = h->maps_ovl_band[1];
  a.ovl_c_lo = h->maps_ovl_c_lo;
  a.ovl_c_hi = h->maps_ovl_c_hi;
  return a;
}

// The preview's detection range compiled as a single-range table set.
int32_t preview_tables(TrikCvHandle* h, PreviewArgs& pa, const TRIK_VIDTRANSCODE_CV_InArgsAlg& range,
                       hipStream_t s, TableSet** set) {
  int32_t rc = acquire_tables(h, &range, 1, s, set);
  if (rc) return rc;
  pa.range = pack_range(range);
  pa.tables = (*set)->d_stripe;
  pa.hue_free = !(*set)->detect.empty() && (*set)->detect[0] != kDetectFull ? 1 : 0;
  return 0;
}


// The line sensor's range in the object sensor's terms: hue 0..359 and
// saturation 0..100 scale to the full 0..255 bytes LSEQ:391-396 fixes.
TRIK_VIDTRANSCODE_CV_InArgsAlg line_alg(int val_from, int val_to) {
  TRIK_VIDTRANSCODE_CV_InArgsAlg r;
  memset(&r, 0, sizeof r);
  r.detectHueFrom = 0;
  r.detectHueTo = 359;
  r.detectSatFrom = 0;
  r.detectSatTo = 100;
  r.detectValFrom = (uint8_t)val_from;
  r.detectValTo = (uint8_t)val_to;
  return r;
}

// LSEQ:391-414: hue and saturation bounds fixed at 0..255 (unscaled), value
// scaled as the object sensor's.
uint32_t scale_val(int v) {
  const int s = (v * 255) / 100;
  return (uint32_t)(s < 0 ? 0 : (s > 255 ? 255 : s));
}
LineArgs line_args(const TrikHsvFrameBatch& b, int val_from, int val_to, int band_start, int band_stop,
                   TrikHsvTargetSums* sums, TrikHsvTarget* targets) {
  LineArgs a;
  a.frames = static_cast<const uint8_t*>(b.frames);
  a.frame_stride = b.frame_stride;
  a.n_frames = b.n_frames;
  a.width = b.width; a.height = b.height; a.line_length = b.line_length;
  a.val_lo = scale_val(val_from);
  a.val_hi = scale_val(val_to);
  a.band_start = band_start;
  a.band_stop = band_stop;
  a.sums = sums;
  a.targets = targets;
  return a;
}

// BitmapBuilder::run's range update (cv_bitmap_builder_reference.hpp:110-130):
// from/to around the centre (hue wraps, sat/val clip), scaled as the webcam's,
// then resetHsvRange (:62-77).
int wrap_value(int v, int adj, int lo, int hi) {  // makeValueWrap, stdcpp.hpp
  v += adj;
  while (v > hi) v -= hi - lo + 1;
  while (v < lo) v += hi - lo + 1;
  return v;
}
int clip_value(int v, int adj, int lo, int hi) {  // makeValueRange, stdcpp.hpp
  v += adj;
  return v > hi ? hi : (v < lo ? lo : v);
}
TRIK_VIDTRANSCODE_CV_InArgsAlg blob_range_args(const TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg& a) {
  TRIK_VIDTRANSCODE_CV_InArgsAlg r;
  memset(&r, 0, sizeof r);
  r.detectHueFrom = (uint16_t)wrap_value(a.detectHue, -(int)a.detectHueTol, 0, 359);
  r.detectHueTo = (uint16_t)wrap_value(a.detectHue, (int)a.detectHueTol, 0, 359);
  r.detectSatFrom = (uint8_t)clip_value(a.detectSat, -(int)a.detectSatTol, 0, 100);
  r.detectSatTo = (uint8_t)clip_value(a.detectSat, (int)a.detectSatTol, 0, 100);
  r.detectValFrom = (uint8_t)clip_value(a.detectVal, -(int)a.detectValTol, 0, 100);
  r.detectValTo = (uint8_t)clip_value(a.detectVal, (int)a.detectValTol, 0, 100);
  return r;  // then the same scaling and wrap packing (WSEQ:425-445 = BMB:62-77)
}

template <typename T>
int32_t grow(T*& p, size_t& cap, size_t bytes) {
  if (bytes <= cap) return 0;
  (void)hipFree(p);
  p = nullptr;
  cap = 0;
  HIP_TRY(hipMalloc(&p, bytes));
  cap = bytes;
  return 0;
}

// Scratch for n frames of W x H.  Stream s waits (device side) for the
// handle's earlier multi-blob work on other streams, which used the same
// scratch; growing it (a larger batch) waits for that work on the host.
int32_t ensure_blob_scratch(TrikCvHandle* h, int n, int w, int hgt, hipStream_t s) {
  const size_t bw = (size_t)(w / 4), bh = (size_t)(hgt / 4), nn = (size_t)(n > 0 ? n : 1);
  const size_t ml = (size_t)blob_max_labels((int)bw, (int)bh);
  if (nn * (bw * bh > 0 ? bw * bh : 1) > h->d_meta_cap || nn * 3 * ml * sizeof(int32_t) > h->d_blob_stats_cap ||
      nn * 24 * sizeof(int32_t) > h->d_blob_top_cap || nn * 8 * sizeof(TrikHsvTarget) > h->d_blob_targets_cap)
    h->blob_users.wait_all();
  HIP_TRY(h->blob_users.order_after(s));
  int32_t r = grow(h->d_meta, h->d_meta_cap, nn * (bw * bh > 0 ? bw * bh : 1));
  // the clusterer's own statistics: zero when allocated, and every clusterer
  // launch leaves the labels it used zero again (blob_ccl_kernel).  The
  // capacity counts only once the zeroing is enqueued, and a failed clusterer
  // launch (which may leave labels non-zero) marks the buffer dirty: the next
  // call zeroes it whole.
  const size_t stats_bytes = nn * 3 * ml * sizeof(int32_t);
  if (!r && (stats_bytes > h->d_blob_stats_cap || h->blob_stats_dirty)) {
    if (stats_bytes > h->d_blob_stats_cap) r = grow(h->d_blob_stats, h->d_blob_stats_cap, stats_bytes);
    if (!r) {
      const hipError_t e = hipMemsetAsync(h->d_blob_stats, 0, h->d_blob_stats_cap, s);
      if (e != hipSuccess) {
        h->blob_stats_dirty = true;
        return fail(TRIK_IVIDTRANSCODE_EFAIL, std::string("hipMemsetAsync(blob stats): ") + hipGetErrorString(e));
      }
      h->blob_stats_dirty = false;
    }
  }
  if (!r) r = grow(h->d_blob_top, h->d_blob_top_cap, nn * 24 * sizeof(int32_t));
  if (!r) r = grow(h->d_blob_targets, h->d_blob_targets_cap, nn * 8 * sizeof(TrikHsvTarget));
  return r;
}

// Compiles the range's tables (cached per handle) and fills the kernel args.
int32_t blob_args(TrikCvHandle* h, const TrikHsvFrameBatch& b, const TRIK_VIDTRANSCODE_CV_InArgsAlg& range,
                  TrikHsvTarget* targets, int32_t* top, uint8_t* meta, uint16_t* labels, int32_t* n_labels,
                  hipStream_t s, BlobArgs& a, TableSet** set) {
  int32_t rc = acquire_tables(h, &range, 1, s, set);
  if (rc) return rc;
  a.frames = static_cast<const uint8_t*>(b.frames);
  a.frame_stride = b.frame_stride;
  a.n_frames = b.n_frames;
  a.width = b.width; a.height = b.height; a.line_length = b.line_length;
  a.range = pack_range(range);
  a.tables = (*set)->d_stripe;
  a.aligned4 = (reinterpret_cast<uintptr_t>(b.frames) & 3) == 0 && (b.n_frames <= 1 || (b.frame_stride & 3) == 0) &&
               (b.line_length & 3) == 0;
  a.meta = meta ? meta : h->d_meta;
  a.labels = labels;
  a.stats = h->d_blob_stats;
  a.max_labels = (int32_t)blob_max_labels(b.width / 4, b.height / 4);
  a.targets = targets ? targets : h->d_blob_targets;
  a.top = top ? top : h->d_blob_top;
  a.n_labels = n_labels;
  return 0;
}

// The multi-blob sensor: the metapixel bitmap on the chroma-run tables of the
// sticky range when the hot-kernel setting allows it (AUTO: batches of at
// least TRIK_HSV_CHROMA_MIN_PIXELS whose exact-path share is low), else the
// stripe-arithmetic kernel inside launch_blob; then the clusterer.
int32_t run_blob(TrikCvHandle* h, BlobArgs& ba, TableSet& t, hipStream_t s) {
  const bool big = (int64_t)ba.n_frames * ba.width * ba.height >= (int64_t)TRIK_HSV_CHROMA_MIN_PIXELS;
  int32_t rc = 0;
  const HotPlan plan = plan_hot(h, t, 0, 1, big, h->hot.load() != TRIK_HSV_HOT_GENERIC && blob_chroma_ok(ba), s, &rc);
  if (rc) return rc;
  ba.meta_ready = 0;
  h->pending_set = nullptr;
  h->hot_groups.assign(1, TRIK_HSV_HOT_STRIPE);
  if (plan == kPlanChroma) {
    HIP_TRY(launch_blob_meta_chroma(ba, t.d_chroma, t.d_tables, s));
    ba.meta_ready = 1;
    h->hot_groups[0] = TRIK_HSV_HOT_CHROMA;
  } else if (plan == kPlanGated) {  // both bitmap kernels, the device runs one (see run_sums)
    BlobArgs bc = ba;
    bc.gate = ba.gate = &t.d_chroma[0].flagged_cost;
    bc.gate_max = ba.gate_max = kChromaMaxCost;
    bc.gate_le = 1;
    ba.gate_le = 0;
    HIP_TRY(launch_blob_meta_chroma(bc, t.d_chroma, t.d_tables, s));
    h->pending_set = &t;
    h->hot_groups[0] = -TRIK_HSV_HOT_STRIPE;
  }
  const int e = launch_blob(ba, s);
  if (e != hipSuccess) {
    h->blob_stats_dirty = true;  // (the clusterer may not have restored its statistics to zero)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, std::string("launch_blob: ") + hipGetErrorString((hipError_t)e));
  }
  return 0;
}

AutoRangeArgs auto_range_args(const TrikHsvFrameBatch& b, uint16_t* out) {
  AutoRangeArgs a;
  a.frames = static_cast<const uint8_t*>(b.frames);
  a.frame_stride = b.frame_stride;
  a.n_frames = b.n_frames;
  a.width = b.width; a.height = b.height; a.line_length = b.line_length; a.layout = b.layout;
  auto_range_zone(b.width, b.height, a.c_lo, a.c_hi, a.r_lo, a.r_hi);
  a.aligned4 = (reinterpret_cast<uintptr_t>(b.frames) & 3) == 0 && (b.n_frames <= 1 || (b.frame_stride & 3) == 0) &&
               (b.line_length & 3) == 0;
  a.out = out;
  return a;
}

}  // namespace

// ---------------------------------------------------------------------------
// Layer 1: XDAIS-shaped quartet
// ---------------------------------------------------------------------------
extern "C" TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_FXNS, TRIK_VIDTRANSCODE_CV_OV7670_FXNS,
    TRIK_VIDTRANSCODE_CV_LINE_FXNS, TRIK_VIDTRANSCODE_CV_WEBCAM_LINE_FXNS;

static const TRIK_IALG_Fxns* table_of(int algo) {
  switch (algo) {
    case kAlgoLine: return &TRIK_VIDTRANSCODE_CV_LINE_FXNS.ialg;
    case kAlgoBlob: return &TRIK_VIDTRANSCODE_CV_OV7670_FXNS.ialg;
    case kAlgoWLine: return &TRIK_VIDTRANSCODE_CV_WEBCAM_LINE_FXNS.ialg;
    default: return &TRIK_VIDTRANSCODE_CV_FXNS.ialg;
  }
}

// A failed init: a handle of TRIK_VIDTRANSCODE_CV_create is deleted; one in
// a framework record keeps a valid object without device resources, because
// the framework calls algFree on it next (TI's ALG_create does), which
// destroys it once.
static void init_failed(TrikCvHandle* h) {
  if (h->owns_memory)
    release(h);
  else
    free_resources(h);
}

// trikCvHandleInit + SetupParams + SetupDynamicParams (WFXNS:146-166) on a
// constructed object; init_failed on failure.
static int32_t init_handle(TrikCvHandle* h, int algo, const TRIK_VIDTRANSCODE_CV_Params* params) {
  if (hipGetDevice(&h->device) != hipSuccess) {
    init_failed(h);
    return fail(TRIK_IALG_EFAIL, "no HIP device");
  }
  h->algo = algo;
  h->params = params ? *params
                     : (algo == kAlgoLine ? k_default_params_line
                                          : (algo == kAlgoBlob ? k_default_params_blob : k_default_params));  // WGLUE:188-191
  // (the webcam line sensor's glue has the webcam object sensor's Params)
  const int32_t rc = setup_dynamic(h, nullptr);      // WFXNS:158-163
  if (rc != TRIK_IALG_EOK) {
    init_failed(h);
    return rc;
  }
  return TRIK_IALG_EOK;
}

static int32_t create_handle(int algo, const TRIK_VIDTRANSCODE_CV_Params* params,
                             TRIK_VIDTRANSCODE_CV_Handle* out_handle) {
  if (!out_handle) return fail(TRIK_IALG_EFAIL, "out_handle is NULL");
  *out_handle = nullptr;
  TrikCvHandle* h = new (std::nothrow) TrikCvHandle();
  if (!h) return fail(TRIK_IALG_EFAIL, "out of memory");
  h->ialg.fxns = table_of(algo);
  const int32_t rc = init_handle(h, algo, params);
  if (rc == TRIK_IALG_EOK) *out_handle = h;
  return rc;
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_create(const TRIK_VIDTRANSCODE_CV_Params* params,
                                               TRIK_VIDTRANSCODE_CV_Handle* out_handle) {
  return create_handle(kAlgoBall, params, out_handle);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_create_line(const TRIK_VIDTRANSCODE_CV_Params* params,
                                                    TRIK_VIDTRANSCODE_CV_Handle* out_handle) {
  return create_handle(kAlgoLine, params, out_handle);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_create_webcam_line(const TRIK_VIDTRANSCODE_CV_Params* params,
                                                           TRIK_VIDTRANSCODE_CV_Handle* out_handle) {
  return create_handle(kAlgoWLine, params, out_handle);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_create_ov7670(const TRIK_VIDTRANSCODE_CV_Params* params,
                                                      TRIK_VIDTRANSCODE_CV_Handle* out_handle) {
  return create_handle(kAlgoBlob, params, out_handle);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_delete(TRIK_VIDTRANSCODE_CV_Handle handle) {
  if (!handle) return fail(TRIK_IALG_EFAIL, "handle is NULL");
  release(handle);
  return TRIK_IALG_EOK;
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_control(TRIK_VIDTRANSCODE_CV_Handle h, int32_t cmd,
                                                TRIK_VIDTRANSCODE_CV_DynamicParams* dyn,
                                                TRIK_IVIDTRANSCODE_Status* status) {
  if (!h || !status) return fail(TRIK_IVIDTRANSCODE_EFAIL, "handle or status is NULL");
  std::lock_guard<std::mutex> lock(h->mu);
  int32_t rc = TRIK_IVIDTRANSCODE_EFAIL;
  status->data.accessMask &= ~((1 << TRIK_XDM_ACCESSMODE_READ) | (1 << TRIK_XDM_ACCESSMODE_WRITE));
  switch (cmd) {  // WFXNS:285-331
    case TRIK_XDM_GETSTATUS:
    case TRIK_XDM_GETBUFINFO:
      status->extendedError = 0;
      status->bufInfo.minNumInBufs = 1;
      status->bufInfo.minNumOutBufs = 1;
      status->bufInfo.minInBufSize[0] = 0;
      status->bufInfo.minOutBufSize[0] = 0;
      set_bit(status->data.accessMask, TRIK_XDM_ACCESSMODE_WRITE);
      rc = TRIK_IVIDTRANSCODE_EOK;
      break;
    case TRIK_XDM_SETPARAMS:
      if (dyn && dyn->base.size == (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_DynamicParams))
        rc = setup_dynamic(h, dyn);
      else
        rc = fail(TRIK_IVIDTRANSCODE_EUNSUPPORTED, "SETPARAMS: dynamic params size mismatch");
      break;
    case TRIK_XDM_RESET:
    case TRIK_XDM_SETDEFAULT:
      rc = setup_dynamic(h, nullptr);
      break;
    case TRIK_XDM_FLUSH:
      rc = TRIK_IVIDTRANSCODE_EOK;
      break;
    case TRIK_XDM_GETVERSION:
      if (status->data.buf && status->data.bufSize >= (int32_t)sizeof k_version) {
        memcpy(status->data.buf, k_version, sizeof k_version);
        set_bit(status->data.accessMask, TRIK_XDM_ACCESSMODE_WRITE);
        rc = TRIK_IVIDTRANSCODE_EOK;
      } else {
        rc = fail(TRIK_IVIDTRANSCODE_EFAIL, "GETVERSION: buffer too small");
      }
      break;
    default:
      rc = fail(TRIK_IVIDTRANSCODE_EFAIL, "unsupported control command");
  }
  return rc;
}

// ---------------------------------------------------------------------------
// Layer 1b: the XDAIS IALG functions and function tables (WFXNS:20-166)
// ---------------------------------------------------------------------------
// algAlloc: one persistent external record for the object (the reference's
// second record, C64x+ on-chip fast RAM, has no use here)
static int32_t ialg_alloc(const TRIK_IALG_Params*, TRIK_IALG_Fxns**, TRIK_IALG_MemRec mem_tab[]) {
  if (!mem_tab) return fail(TRIK_IALG_EFAIL, "algAlloc: mem_tab is NULL");
  mem_tab[0].size = (uint32_t)sizeof(TrikCvHandle);
  mem_tab[0].alignment = (int32_t)alignof(TrikCvHandle);
  mem_tab[0].space = TRIK_IALG_EXTERNAL;
  mem_tab[0].attrs = TRIK_IALG_PERSIST;
  mem_tab[0].base = nullptr;
  return 1;
}

// algInit: the object is constructed in the framework's record; the fxns
// word the framework stored there is kept
static int32_t ialg_init(int algo, TRIK_IALG_Handle alg, const TRIK_IALG_MemRec mem_tab[], const TRIK_IALG_Params* params) {
  if (!alg || !mem_tab || mem_tab[0].base != (void*)alg)
    return fail(TRIK_IALG_EFAIL, "algInit: the handle must be mem_tab[0].base");
  if (mem_tab[0].size < sizeof(TrikCvHandle) || (reinterpret_cast<uintptr_t>(alg) % alignof(TrikCvHandle)))
    return fail(TRIK_IALG_EFAIL, "algInit: mem_tab[0] smaller or less aligned than algAlloc asked");
  if (params && params->size != (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_Params))
    return fail(TRIK_IALG_EFAIL, "algInit: params size mismatch");
  const TRIK_IALG_Fxns* fxns = alg->fxns;
  TrikCvHandle* h = new (alg) TrikCvHandle();
  h->ialg.fxns = fxns ? fxns : table_of(algo);
  h->owns_memory = false;
  return init_handle(h, algo, reinterpret_cast<const TRIK_VIDTRANSCODE_CV_Params*>(params));
}

static int32_t ialg_init_ball(TRIK_IALG_Handle a, const TRIK_IALG_MemRec* m, TRIK_IALG_Handle, const TRIK_IALG_Params* p) {
  return ialg_init(kAlgoBall, a, m, p);
}
static int32_t ialg_init_blob(TRIK_IALG_Handle a, const TRIK_IALG_MemRec* m, TRIK_IALG_Handle, const TRIK_IALG_Params* p) {
  return ialg_init(kAlgoBlob, a, m, p);
}
static int32_t ialg_init_line(TRIK_IALG_Handle a, const TRIK_IALG_MemRec* m, TRIK_IALG_Handle, const TRIK_IALG_Params* p) {
  return ialg_init(kAlgoLine, a, m, p);
}
static int32_t ialg_init_wline(TRIK_IALG_Handle a, const TRIK_IALG_MemRec* m, TRIK_IALG_Handle, const TRIK_IALG_Params* p) {
  return ialg_init(kAlgoWLine, a, m, p);
}

// algFree: the object is destroyed; its record is returned for the framework
static int32_t ialg_free(TRIK_IALG_Handle alg, TRIK_IALG_MemRec mem_tab[]) {
  if (!alg || !mem_tab) return fail(TRIK_IALG_EFAIL, "algFree: NULL argument");
  TrikCvHandle* h = reinterpret_cast<TrikCvHandle*>(alg);
  if (h->owns_memory) return fail(TRIK_IALG_EFAIL, "algFree: handle made by TRIK_VIDTRANSCODE_CV_create");
  release(h);
  mem_tab[0].base = alg;
  mem_tab[0].size = (uint32_t)sizeof(TrikCvHandle);
  mem_tab[0].alignment = (int32_t)alignof(TrikCvHandle);
  mem_tab[0].space = TRIK_IALG_EXTERNAL;
  mem_tab[0].attrs = TRIK_IALG_PERSIST;
  return 1;
}

static int32_t xdais_process(TRIK_IALG_Handle alg, TRIK_XDM1_BufDesc* in, TRIK_XDM_BufDesc* out,
                             TRIK_IVIDTRANSCODE_InArgs* in_args, TRIK_IVIDTRANSCODE_OutArgs* out_args) {
  return TRIK_VIDTRANSCODE_CV_process(reinterpret_cast<TRIK_VIDTRANSCODE_CV_Handle>(alg), in, out,
                                      reinterpret_cast<TRIK_VIDTRANSCODE_CV_InArgs*>(in_args),
                                      reinterpret_cast<TRIK_VIDTRANSCODE_CV_OutArgs*>(out_args));
}

static int32_t xdais_control(TRIK_IALG_Handle alg, int32_t cmd, TRIK_VIDTRANSCODE_CV_DynamicParams* dyn,
                             TRIK_IVIDTRANSCODE_Status* status) {
  return TRIK_VIDTRANSCODE_CV_control(reinterpret_cast<TRIK_VIDTRANSCODE_CV_Handle>(alg), cmd, dyn, status);
}

// WFXNS:20-29: module ID, activate, alloc, control, deactivate, free, init,
// moved, numAlloc (NULL => IALG_MAXMEMRECS)
#define TRIK_IALGFXNS(self, init) {&self, nullptr, ialg_alloc, nullptr, nullptr, ialg_free, init, nullptr, nullptr}

extern "C" {
TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_FXNS = {TRIK_IALGFXNS(TRIK_VIDTRANSCODE_CV_FXNS, ialg_init_ball),
                                                     xdais_process, xdais_control};
TRIK_IALG_Fxns TRIK_VIDTRANSCODE_CV_IALG = TRIK_IALGFXNS(TRIK_VIDTRANSCODE_CV_FXNS, ialg_init_ball);
TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_OV7670_FXNS = {
    TRIK_IALGFXNS(TRIK_VIDTRANSCODE_CV_OV7670_FXNS, ialg_init_blob), xdais_process, xdais_control};
TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_LINE_FXNS = {TRIK_IALGFXNS(TRIK_VIDTRANSCODE_CV_LINE_FXNS, ialg_init_line),
                                                          xdais_process, xdais_control};
TRIK_IVIDTRANSCODE_Fxns TRIK_VIDTRANSCODE_CV_WEBCAM_LINE_FXNS = {
    TRIK_IALGFXNS(TRIK_VIDTRANSCODE_CV_WEBCAM_LINE_FXNS, ialg_init_wline), xdais_process, xdais_control};
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_alloc(const TRIK_IALG_Params* params, TRIK_IALG_Fxns** parent_fxns,
                                              TRIK_IALG_MemRec mem_tab[]) {
  return ialg_alloc(params, parent_fxns, mem_tab);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_initObj(TRIK_IALG_Handle alg, const TRIK_IALG_MemRec mem_tab[],
                                                TRIK_IALG_Handle parent, const TRIK_IALG_Params* params) {
  return ialg_init_ball(alg, mem_tab, parent, params);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_free(TRIK_IALG_Handle alg, TRIK_IALG_MemRec mem_tab[]) {
  return ialg_free(alg, mem_tab);
}

extern "C" int32_t TRIK_VIDTRANSCODE_CV_process(TRIK_VIDTRANSCODE_CV_Handle h,
                                                TRIK_XDM1_BufDesc* in_bufs,
                                                TRIK_XDM_BufDesc* out_bufs,
                                                TRIK_VIDTRANSCODE_CV_InArgs* in_args,
                                                TRIK_VIDTRANSCODE_CV_OutArgs* out_args) {
  if (!h || !in_bufs || !out_bufs || !in_args || !out_args)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "NULL argument");
  std::lock_guard<std::mutex> lock(h->mu);
  const bool blob = h->algo == kAlgoBlob;  // the ov7670 object sensor's own InArgs / OutArgs
  const int32_t in_want = blob ? (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_OV7670_InArgs)
                               : (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_InArgs);
  const int32_t out_want = blob ? (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_OV7670_OutArgs)
                                : (int32_t)sizeof(TRIK_VIDTRANSCODE_CV_OutArgs);
  if (in_args->base.size != in_want ||  // WFXNS:192-197
      out_args->base.size != out_want) {
    set_bit(out_args->base.extendedError, TRIK_XDM_UNSUPPORTEDPARAM_BIT);
    return fail(TRIK_IVIDTRANSCODE_EUNSUPPORTED, "InArgs/OutArgs size mismatch");
  }
  if (in_bufs->numBufs != 1 || out_bufs->numBufs < h->params.base.numOutputStreams) {  // :199-204
    set_bit(out_args->base.extendedError, TRIK_XDM_UNSUPPORTEDPARAM_BIT);
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "buffer count");
  }
  TRIK_XDM1_SingleBufDesc* in = &in_bufs->descs[0];
  if (!in->buf || in_args->base.numBytes < 0 || in_args->base.numBytes > in->bufSize) {  // :207-214
    set_bit(out_args->base.extendedError, TRIK_XDM_UNSUPPORTEDPARAM_BIT);
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "input buffer");
  }
  set_bit(in->accessMask, TRIK_XDM_ACCESSMODE_READ);  // :216-221
  out_args->base.bitsConsumed = in_args->base.numBytes * CHAR_BIT;
  out_args->base.decodedPictureType = -1;       // IVIDEO_NA_PICTURE
  out_args->base.decodedPictureStructure = -1;  // IVIDEO_CONTENTTYPE_NA
  out_args->base.decodedHeight = h->dyn.inputHeight;
  out_args->base.decodedWidth = h->dyn.inputWidth;
  const int64_t in_size = in_args->base.numBytes;

  TRIK_XDM1_SingleBufDesc* out = nullptr;
  int8_t* out_ptr = nullptr;
  int64_t out_size = 0;
  if (h->params.base.numOutputStreams == 1) {  // :226-235
    out = &out_args->base.encodedBuf[0];
    out->buf = out_bufs->bufs ? out_bufs->bufs[0] : nullptr;
    out->bufSize = out_bufs->bufSizes ? out_bufs->bufSizes[0] : 0;
    out->accessMask = 0;
    out_ptr = out->buf;
    out_size = out->bufSize;
    if (out_ptr && out_size > 0) memset(out_ptr, 0, (size_t)out_size);
  }

  // trikCvProceedImage + BallDetector::run (WGLUE:291-320, WSEQ:412-508)
  int32_t rc = TRIK_IVIDTRANSCODE_EOK;
  std::string why;
  if (!h->alg_ready) {
    rc = TRIK_IVIDTRANSCODE_EFAIL; why = "CV algorithm not created";
  } else if ((int64_t)h->in_h * h->in_ll > in_size ||
             (h->layout == TRIK_HSV_LAYOUT_OV7670 && 2LL * h->in_h * h->in_ll > in_size)) {
    rc = TRIK_IVIDTRANSCODE_EFAIL; why = "input buffer smaller than the image";  // WSEQ:415-416
  } else if ((int64_t)h->out_h * h->out_ll > out_size) {
    rc = TRIK_IVIDTRANSCODE_EFAIL; why = "output buffer smaller than the preview";  // WSEQ:417-418
  }
  if (rc == TRIK_IVIDTRANSCODE_EOK) {
    out_size = (int64_t)h->out_h * h->out_ll;  // WSEQ:419
    TRIK_VIDTRANSCODE_CV_OutArgsAlg& oa = out_args->alg;
    auto* ia7 = reinterpret_cast<const TRIK_VIDTRANSCODE_CV_OV7670_InArgs*>(in_args);
    auto* oa7 = reinterpret_cast<TRIK_VIDTRANSCODE_CV_OV7670_OutArgs*>(out_args);
    if (blob)
      memset(oa7->alg.target, 0, sizeof oa7->alg.target);  // OSEQ:563
    else {
      oa.targetX = 0; oa.targetY = 0; oa.targetSize = 0;
    }
    if (h->in_w > 0 && h->in_h > 0) {
      int prev = 0;
      const bool switched = hipGetDevice(&prev) == hipSuccess && prev != h->device;
      if (switched) (void)hipSetDevice(h->device);
      const size_t fb = (size_t)h->in_h * h->in_ll * (h->layout == TRIK_HSV_LAYOUT_OV7670 ? 2 : 1);
      auto body = [&]() -> int32_t {
        if (!h->stream) HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        if (fb > h->d_frame_cap) {
          (void)hipFree(h->d_frame);
          h->d_frame = nullptr; h->d_frame_cap = 0;
          HIP_TRY(hipMalloc(&h->d_frame, fb));
          h->d_frame_cap = fb;
        }
        if (!h->d_sums) HIP_TRY(hipMalloc(&h->d_sums, sizeof(TrikHsvTargetSums)));
        if (!h->d_targets) HIP_TRY(hipMalloc(&h->d_targets, sizeof(TrikHsvTarget)));
        HIP_TRY(hipMemcpyAsync(h->d_frame, in->buf, fb, hipMemcpyHostToDevice, h->stream));
        TrikHsvFrameBatch b = {h->d_frame, (int64_t)fb, 1, h->in_w, h->in_h, h->in_ll, h->layout};
        HIP_TRY(hipMemsetAsync(h->d_sums, 0, sizeof(TrikHsvTargetSums), h->stream));
        if (blob) {  // BallDetector<YUV422P>::run, OSEQ:516-602
          if (ia7->alg.setHsvRange) h->blob_range = blob_range_args(ia7->alg);  // BMB:110-130
          int32_t r = ensure_blob_scratch(h, 1, h->in_w, h->in_h, h->stream);
          if (r) return r;
          BlobArgs ba;
          TableSet* set = nullptr;
          r = blob_args(h, b, h->blob_range, nullptr, nullptr, nullptr, nullptr, nullptr, h->stream, ba, &set);
          if (r) return r;
          r = run_blob(h, ba, *set, h->stream);
          if (r) return r;
          r = note_uses(h, set, false, h->stream, &h->blob_users);
          if (r) return r;
          if (out_ptr && out_size > 0) {  // preview: set metapixels, guide lines, target marks
            const size_t pb = (size_t)out_size;
            r = grow(h->d_preview, h->d_preview_cap, pb);
            if (r) return r;
            r = ensure_maps(h, h->in_w, h->in_h, h->out_w, h->out_h, h->stream);
            if (r) return r;
            TRIK_VIDTRANSCODE_CV_InArgsAlg none;
            memset(&none, 0, sizeof none);
            PreviewArgs pa = preview_args(h, b, none, h->out_w, h->out_h, h->out_ll, h->d_preview, (int64_t)pb);
            pa.meta = ba.meta;
            HIP_TRY(launch_preview_body(pa, h->stream));
            HIP_TRY(launch_blob_overlay(pa, ba.top, h->stream));
            r = note_uses(h, nullptr, true, h->stream);
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(out_ptr, h->d_preview, pb, hipMemcpyDeviceToHost, h->stream));
          }
          TrikHsvTarget t[8];
          HIP_TRY(hipMemcpyAsync(t, ba.targets, sizeof t, hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(hipStreamSynchronize(h->stream));
          for (int i = 0; i < 8; ++i) {
            oa7->alg.target[i].x = t[i].x;
            oa7->alg.target[i].y = t[i].y;
            oa7->alg.target[i].size = t[i].size;
          }
          // autoDetectHsv: the ov7670 range detector is a simulated annealing
          // seeded by srand(time(NULL)) -- not reproducible; detect* untouched.
          return 0;
        }
        if (h->algo == kAlgoLine) {  // LineDetector::run, LSEQ:376-476
          const TRIK_VIDTRANSCODE_CV_InArgsAlg& ia = in_args->alg;
          HIP_TRY(launch_line(line_args(b, ia.detectValFrom, ia.detectValTo, h->line_band[0],
                                        h->line_band[1], h->d_sums, h->d_targets), h->stream));
          if (out_ptr && out_size > 0) {  // preview: window columns only, then the overlays
            const size_t pb = (size_t)out_size;
            if (pb > h->d_preview_cap) {
              (void)hipFree(h->d_preview);
              h->d_preview = nullptr; h->d_preview_cap = 0;
              HIP_TRY(hipMalloc(&h->d_preview, pb));
              h->d_preview_cap = pb;
            }
            int32_t r = ensure_maps(h, h->in_w, h->in_h, h->out_w, h->out_h, h->stream, 5, h->in_w - 5);
            if (r) return r;
            PreviewArgs pa = preview_args(h, b, ia, h->out_w, h->out_h, h->out_ll, h->d_preview, (int64_t)pb);
            TableSet* set = nullptr;
            r = preview_tables(h, pa, line_alg(ia.detectValFrom, ia.detectValTo), h->stream, &set);
            if (r) return r;
            HIP_TRY(launch_line_preview(pa, h->d_sums, 1, h->stream));
            r = note_uses(h, set, true, h->stream);
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(out_ptr, h->d_preview, pb, hipMemcpyDeviceToHost, h->stream));
          }
          TrikHsvTarget t;
          HIP_TRY(hipMemcpyAsync(&t, h->d_targets, sizeof t, hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(hipStreamSynchronize(h->stream));
          oa.targetX = t.x; oa.targetY = t.y; oa.targetSize = t.size;
          // autoDetectHsv: the line sensor's range detector is a simulated
          // annealing seeded by srand(time(NULL)) -- not reproducible; detect*
          // are left untouched.
          h->line_band[0] = h->in_h / 2;  // LSEQ:449-450, read by the next run
          h->line_band[1] = h->in_h / 2 + 80;
          return 0;
        }
        if (h->algo == kAlgoWLine) {  // webcam LineDetector::run, LSEQW:330-420
          // hue and saturation fixed to the full bytes, V from InArgs (LSEQW:345-351)
          const TRIK_VIDTRANSCODE_CV_InArgsAlg wr = line_alg(in_args->alg.detectValFrom, in_args->alg.detectValTo);
          int32_t r = run_sums(h, &b, &wr, 1, h->d_sums, nullptr, h->stream);
          if (r) return r;
          HIP_TRY(launch_wline_targets(1, h->in_w, h->in_h, h->d_sums, h->d_targets, h->stream));
          if (out_ptr && out_size > 0) {  // every pixel (LSEQW:232-269), then the thin and target lines
            const size_t pb = (size_t)out_size;
            r = grow(h->d_preview, h->d_preview_cap, pb);
            if (r) return r;
            r = ensure_maps(h, h->in_w, h->in_h, h->out_w, h->out_h, h->stream);
            if (r) return r;
            PreviewArgs pa = preview_args(h, b, wr, h->out_w, h->out_h, h->out_ll, h->d_preview, (int64_t)pb);
            TableSet* set = nullptr;
            r = preview_tables(h, pa, wr, h->stream, &set);
            if (r) return r;
            HIP_TRY(launch_line_preview(pa, h->d_sums, 0, h->stream));
            r = note_uses(h, set, true, h->stream);
            if (r) return r;
            HIP_TRY(hipMemcpyAsync(out_ptr, h->d_preview, pb, hipMemcpyDeviceToHost, h->stream));
          }
          TrikHsvTarget t;
          HIP_TRY(hipMemcpyAsync(&t, h->d_targets, sizeof t, hipMemcpyDeviceToHost, h->stream));
          HIP_TRY(hipStreamSynchronize(h->stream));
          oa.targetX = t.x; oa.targetY = t.y; oa.targetSize = t.size;
          // autoDetectHsv: this sensor's range detector is a simulated annealing
          // seeded by srand(time(NULL)) (its cv_hsv_range_detector.hpp:200) --
          // not reproducible; detect* are left untouched.
          return 0;
        }
        int32_t r = run_sums(h, &b, &in_args->alg, 1, h->d_sums, nullptr, h->stream);
        if (r) return r;
        HIP_TRY(launch_targets(b, 1, h->d_sums, h->d_targets, h->stream));
        uint16_t detect[6] = {0, 0, 0, 0, 0, 0};
        const bool auto_detect = in_args->alg.autoDetectHsv != 0;
        if (auto_detect) {  // WSEQ:455-462
          if (!h->d_auto) HIP_TRY(hipMalloc(&h->d_auto, 6 * sizeof(uint16_t)));
          HIP_TRY(launch_auto_range(auto_range_args(b, h->d_auto), h->stream));
          HIP_TRY(hipMemcpyAsync(detect, h->d_auto, sizeof detect, hipMemcpyDeviceToHost, h->stream));
        }
        if (out_ptr && out_size > 0) {  // the preview stream (WSEQ:316-354, 471-494)
          const size_t pb = (size_t)out_size;
          if (pb > h->d_preview_cap) {
            (void)hipFree(h->d_preview);
            h->d_preview = nullptr; h->d_preview_cap = 0;
            HIP_TRY(hipMalloc(&h->d_preview, pb));
            h->d_preview_cap = pb;
          }
          r = ensure_maps(h, h->in_w, h->in_h, h->out_w, h->out_h, h->stream);
          if (r) return r;
          PreviewArgs pa = preview_args(h, b, in_args->alg, h->out_w, h->out_h, h->out_ll, h->d_preview,
                                        (int64_t)pb);
          TableSet* set = nullptr;
          r = preview_tables(h, pa, in_args->alg, h->stream, &set);
          if (r) return r;
          HIP_TRY(launch_preview(pa, h->d_sums, 1, h->stream));
          r = note_uses(h, set, true, h->stream);
          if (r) return r;
          HIP_TRY(hipMemcpyAsync(out_ptr, h->d_preview, pb, hipMemcpyDeviceToHost, h->stream));
        }
        TrikHsvTarget t;
        HIP_TRY(hipMemcpyAsync(&t, h->d_targets, sizeof t, hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        oa.targetX = t.x; oa.targetY = t.y; oa.targetSize = t.size;
        if (auto_detect) {
          oa.detectHue = detect[0]; oa.detectHueTolerance = detect[1];
          oa.detectSat = detect[2]; oa.detectSatTolerance = detect[3];
          oa.detectVal = detect[4]; oa.detectValTolerance = detect[5];
        }
        return 0;
      };
      const int32_t r = body();
      if (switched) (void)hipSetDevice(prev);
      if (r) { rc = TRIK_IVIDTRANSCODE_EFAIL; why = g_last_error; }
    }
    // OutArgs.detect* are written only when autoDetectHsv is set (WSEQ:455-462)
  }
  if (rc != TRIK_IVIDTRANSCODE_EOK) {
    set_bit(out_args->base.extendedError, TRIK_XDM_CORRUPTEDDATA_BIT);  // WFXNS:243-247
    return fail(rc, why);
  }
  if (out) {  // WFXNS:249-259
    out->bufSize = (int32_t)out_size;
    set_bit(out->accessMask, TRIK_XDM_ACCESSMODE_WRITE);
    out_args->base.bitsGenerated[0] = out->bufSize * CHAR_BIT;
    out_args->base.encodedPictureType[0] = out_args->base.decodedPictureType;
    out_args->base.encodedPictureStructure[0] = out_args->base.decodedPictureStructure;
    out_args->base.outputID[0] = in_args->base.inputID;
    out_args->base.inputFrameSkipTranscodeFlag[0] = 0;
  }
  out_args->base.outBufsInUseFlag = 0;
  return TRIK_IVIDTRANSCODE_EOK;
}

// ---------------------------------------------------------------------------
// Layer 2: batched device API
// ---------------------------------------------------------------------------
namespace {

// A batched call runs on the handle's device (one thread may drive several
// GPUs, one handle each); the caller's current device is restored after.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    int cur = 0;
    if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// A device buffer handed to a batched call must be device-accessible memory
// of the handle's device ("" if so).
std::string device_buffer_error(const void* p, int dev, const char* what) {
  if (!p) return "";
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return std::string(what) + " is not device-accessible memory";
  }
  if (at.type == hipMemoryTypeUnregistered)
    return std::string(what) + " is pageable host memory, not device-accessible memory";
  if (at.type == hipMemoryTypeDevice && at.device != dev)
    return std::string(what) + " is on device " + std::to_string(at.device) + ", the handle on device " +
           std::to_string(dev);
  return "";
}

}  // namespace

extern "C" int32_t trik_hsv_set_hot_kernel(TRIK_VIDTRANSCODE_CV_Handle h, int32_t kind) {
  if (!h || kind < TRIK_HSV_HOT_AUTO || kind > TRIK_HSV_HOT_GENERIC) return -1;
  return h->hot.exchange(kind);
}

extern "C" int32_t trik_hsv_set_reserved_cus(TRIK_VIDTRANSCODE_CV_Handle h, int32_t n) {
  if (!h || n < 0 || n > 32) return -1;
  return h->reserved_cus.exchange(n);
}

extern "C" int32_t trik_hsv_last_hot_kernel(TRIK_VIDTRANSCODE_CV_Handle h) {
  if (!h) return 0;
  std::lock_guard<std::mutex> lock(h->mu);
  {
    DeviceGuard dg(h->device);
    resolve_pending(h);
  }
  int kind = 0;
  for (int8_t k : h->hot_groups) {
    if (!k) continue;
    kind = kind == 0 || kind == k ? k : TRIK_HSV_HOT_MIXED;
  }
  return kind;
}

extern "C" int32_t trik_hsv_chroma_share(TRIK_VIDTRANSCODE_CV_Handle h, double* share) {
  if (!h || !share) return fail(TRIK_IVIDTRANSCODE_EFAIL, "NULL handle or share");
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  TableSet* t = h->sums_set;
  *share = -1.0;
  if (t && t->chroma_built) {
    HIP_TRY(hipEventSynchronize(t->cost_ready));
    *share = t->share();
  }
  return 0;
}

extern "C" int32_t trik_hsv_chroma_measured_share(TRIK_VIDTRANSCODE_CV_Handle h, double* share) {
  if (!h || !share) return fail(TRIK_IVIDTRANSCODE_EFAIL, "NULL handle or share");
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  TableSet* t = h->sums_set;
  *share = -1.0;
  if (!t) return 0;
  if (t->words_pending) HIP_TRY(hipEventSynchronize(t->words_ready));
  poll_measured(*t);
  for (const TableSet::Probe& p : t->probes)
    if (p.measured > *share) *share = p.measured;
  return 0;
}

extern "C" const char* trik_hsv_version(void) { return "trik-hsv-mi355x 0.1.0 (gfx950)"; }

extern "C" const char* trik_hsv_last_error(void) { return g_last_error.c_str(); }

// The batch's frames and the output buffer live on the handle's device.
static int32_t check_device(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b, const void* out) {
  if (!b || b->n_frames <= 0) return 0;
  DeviceGuard dg(h->device);
  std::string e = device_buffer_error(b->frames, h->device, "frames");
  if (e.empty()) e = device_buffer_error(out, h->device, "the output buffer");
  return e.empty() ? 0 : fail(TRIK_IVIDTRANSCODE_EFAIL, e);
}

static int32_t check_common(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                            const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n,
                            const void* sums) {
  if (!h) return fail(TRIK_IVIDTRANSCODE_EFAIL, "handle is NULL");
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (n < 1 || n > TRIK_HSV_MAX_RANGES || !ranges)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "n_ranges must be 1..64");
  if (!sums && b->n_frames > 0) return fail(TRIK_IVIDTRANSCODE_EFAIL, "sums is NULL");
  return check_device(h, b, sums);
}

extern "C" int32_t trik_hsv_batch_sums(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                       const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n,
                                       TrikHsvTargetSums* sums, void* stream) {
  int32_t rc = check_common(h, b, ranges, n, sums);
  if (rc) return rc;
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  return run_sums(h, b, ranges, n, sums, nullptr, static_cast<hipStream_t>(stream));
}

extern "C" int32_t trik_hsv_batch_totals(int32_t n_frames, int32_t n_ranges, const TrikHsvTargetSums* sums,
                                         TrikHsvTargetSums* totals, void* stream) {
  if (n_frames < 0 || n_ranges < 1 || n_ranges > TRIK_HSV_MAX_RANGES)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "batch_totals: need n_frames >= 0 and n_ranges 1..64");
  if (!totals || (n_frames > 0 && !sums)) return fail(TRIK_IVIDTRANSCODE_EFAIL, "batch_totals: NULL buffer");
  HIP_TRY(launch_totals(n_frames, n_ranges, sums, totals, static_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int32_t trik_hsv_batch_targets(const TrikHsvFrameBatch* b, int32_t n,
                                          const TrikHsvTargetSums* sums, TrikHsvTarget* targets,
                                          void* stream) {
  // only the geometry matters here (no frame bytes are read)
  if (!b) return fail(TRIK_IVIDTRANSCODE_EFAIL, "batch is NULL");
  if (b->n_frames < 0 || b->width <= 0 || b->height <= 0 || b->width > 32767 || b->height > 32767)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "batch_targets: need n_frames >= 0 and 0 < width, height <= 32767");
  if (n < 1 || n > TRIK_HSV_MAX_RANGES) return fail(TRIK_IVIDTRANSCODE_EFAIL, "n_ranges must be 1..64");
  if (b->n_frames > 0 && (!sums || !targets)) return fail(TRIK_IVIDTRANSCODE_EFAIL, "NULL buffer");
  HIP_TRY(launch_targets(*b, n, sums, targets, static_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int32_t trik_hsv_process_batch(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                          const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n,
                                          TrikHsvTargetSums* sums, TrikHsvTarget* targets,
                                          void* stream) {
  int32_t rc = check_common(h, b, ranges, n, sums);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  StepOut step;
  step.targets = targets;
  return run_sums(h, b, ranges, n, sums, nullptr, s, &step);
}

extern "C" int32_t trik_hsv_process_batch_totals(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                                 const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n,
                                                 TrikHsvTargetSums* sums, TrikHsvTarget* targets,
                                                 TrikHsvTargetSums* totals, void* stream) {
  int32_t rc = check_common(h, b, ranges, n, sums);
  if (rc) return rc;
  if (!totals) return fail(TRIK_IVIDTRANSCODE_EFAIL, "totals is NULL");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  rc = check_device(h, b, totals);
  if (rc) return rc;
  StepOut step;
  step.targets = targets;
  step.totals = totals;
  return run_sums(h, b, ranges, n, sums, nullptr, s, &step);
}

extern "C" int32_t trik_hsv_batch_masks(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                        const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n,
                                        uint8_t* masks, TrikHsvTargetSums* sums, void* stream) {
  int32_t rc = check_common(h, b, ranges, n, sums);
  if (rc) return rc;
  if (n > 8) return fail(TRIK_IVIDTRANSCODE_EFAIL, "mask mode supports at most 8 ranges");
  if (!masks && b->n_frames > 0) return fail(TRIK_IVIDTRANSCODE_EFAIL, "masks is NULL");
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  return run_sums(h, b, ranges, n, sums, masks, static_cast<hipStream_t>(stream));
}

extern "C" int32_t trik_hsv_batch_preview(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                          const TRIK_VIDTRANSCODE_CV_InArgsAlg* range,
                                          const TrikHsvTargetSums* sums, int32_t sums_pitch,
                                          int32_t out_width, int32_t out_height,
                                          int32_t out_line_length, uint8_t* previews,
                                          int64_t preview_stride, void* stream) {
  int32_t rc = check_common(h, b, range, 1, sums);
  if (rc) return rc;
  if (out_width < 0 || out_height < 0 || out_line_length < 2 * out_width || sums_pitch < 1)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "preview geometry: need out_line_length >= 2*out_width, sums_pitch >= 1");
  const int64_t pb = (int64_t)out_height * out_line_length;
  if (b->n_frames > 1 && preview_stride < pb)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "preview_stride smaller than one preview");
  if (!previews && b->n_frames > 0 && pb > 0) return fail(TRIK_IVIDTRANSCODE_EFAIL, "previews is NULL");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  if (b->n_frames == 0 || pb == 0) return 0;
  rc = check_device(h, b, previews);
  if (rc) return rc;
  // the preview kernel writes every byte of each preview, zeros included (WFXNS:234)
  rc = ensure_maps(h, b->width, b->height, out_width, out_height, s);
  if (rc) return rc;
  PreviewArgs pa = preview_args(h, *b, *range, out_width, out_height, out_line_length, previews, preview_stride);
  TableSet* set = nullptr;
  rc = preview_tables(h, pa, *range, s, &set);
  if (rc) return rc;
  HIP_TRY(launch_preview(pa, sums, sums_pitch, s));
  return note_uses(h, set, true, s);
}

extern "C" int32_t trik_hsv_batch_auto_range(const TrikHsvFrameBatch* b, uint16_t* out, void* stream) {
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (!out && b->n_frames > 0) return fail(TRIK_IVIDTRANSCODE_EFAIL, "out is NULL");
  HIP_TRY(launch_auto_range(auto_range_args(*b, out), static_cast<hipStream_t>(stream)));
  return 0;
}

extern "C" int32_t trik_hsv_line_batch(const TrikHsvFrameBatch* b, int32_t val_from, int32_t val_to,
                                       int32_t band_start, int32_t band_stop, TrikHsvTargetSums* sums,
                                       TrikHsvTarget* targets, void* stream) {
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (b->layout != TRIK_HSV_LAYOUT_OV7670)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "the line sensor takes the ov7670 layout (YUV422P)");
  if (b->n_frames > 0 && !sums) return fail(TRIK_IVIDTRANSCODE_EFAIL, "sums is NULL");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (b->n_frames == 0) return 0;
  HIP_TRY(hipMemsetAsync(sums, 0, sizeof(TrikHsvTargetSums) * (size_t)b->n_frames, s));
  if (b->width == 0 || b->height == 0) {
    if (targets) HIP_TRY(hipMemsetAsync(targets, 0, sizeof(TrikHsvTarget) * (size_t)b->n_frames, s));
    return 0;
  }
  HIP_TRY(launch_line(line_args(*b, val_from, val_to, band_start, band_stop, sums, targets), s));
  return 0;
}

extern "C" int32_t trik_hsv_line_preview(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                         int32_t val_from, int32_t val_to, const TrikHsvTargetSums* sums,
                                         int32_t out_width, int32_t out_height, int32_t out_line_length,
                                         uint8_t* previews, int64_t preview_stride, void* stream) {
  if (!h) return fail(TRIK_IVIDTRANSCODE_EFAIL, "handle is NULL");
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (b->layout != TRIK_HSV_LAYOUT_OV7670)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "the line sensor takes the ov7670 layout (YUV422P)");
  if (out_width < 0 || out_height < 0 || out_line_length < 2 * out_width)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "preview geometry: need out_line_length >= 2*out_width");
  const int64_t pb = (int64_t)out_height * out_line_length;
  if (b->n_frames > 1 && preview_stride < pb)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "preview_stride smaller than one preview");
  if (b->n_frames > 0 && pb > 0 && (!previews || !sums)) return fail(TRIK_IVIDTRANSCODE_EFAIL, "NULL buffer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  if (b->n_frames == 0 || pb == 0) return 0;
  int32_t rc = check_device(h, b, previews);
  if (rc) return rc;
  rc = ensure_maps(h, b->width, b->height, out_width, out_height, s, 5, b->width - 5);
  if (rc) return rc;
  TRIK_VIDTRANSCODE_CV_InArgsAlg ia;
  memset(&ia, 0, sizeof ia);
  PreviewArgs pa = preview_args(h, *b, ia, out_width, out_height, out_line_length, previews, preview_stride);
  TableSet* set = nullptr;
  rc = preview_tables(h, pa, line_alg(val_from, val_to), s, &set);
  if (rc) return rc;
  HIP_TRY(launch_line_preview(pa, sums, 1, s));
  return note_uses(h, set, true, s);
}

extern "C" int32_t trik_hsv_blob_batch(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                       const TRIK_VIDTRANSCODE_CV_OV7670_InArgsAlg* hsv, TrikHsvTarget* targets,
                                       int32_t* top, uint8_t* meta, uint16_t* labels, int32_t* n_labels,
                                       void* stream) {
  if (!h) return fail(TRIK_IVIDTRANSCODE_EFAIL, "handle is NULL");
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (b->layout != TRIK_HSV_LAYOUT_OV7670)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "the multi-blob sensor takes the ov7670 layout (YUV422P)");
  if (!hsv) return fail(TRIK_IVIDTRANSCODE_EFAIL, "hsv is NULL");
  if (b->width % 32 || b->height % 4) return fail(TRIK_IVIDTRANSCODE_EFAIL, "width % 32 / height % 4");
  if (b->width > 8192 || blob_max_labels(b->width / 4, b->height / 4) > 30000)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "frame too large for the multi-blob sensor");
  if (b->n_frames > 0 && !targets) return fail(TRIK_IVIDTRANSCODE_EFAIL, "targets is NULL");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  if (b->n_frames == 0) return 0;
  int32_t r = check_device(h, b, targets);
  if (r) return r;
  if (b->width == 0 || b->height == 0) {
    HIP_TRY(hipMemsetAsync(targets, 0, sizeof(TrikHsvTarget) * 8 * (size_t)b->n_frames, s));
    if (top) HIP_TRY(hipMemsetAsync(top, 0, sizeof(int32_t) * 24 * (size_t)b->n_frames, s));
    if (n_labels) HIP_TRY(hipMemsetAsync(n_labels, 0, sizeof(int32_t) * (size_t)b->n_frames, s));
    return 0;
  }
  r = ensure_blob_scratch(h, b->n_frames, b->width, b->height, s);
  if (r) return r;
  BlobArgs ba;
  TableSet* set = nullptr;
  r = blob_args(h, *b, blob_range_args(*hsv), targets, top, meta, labels, n_labels, s, ba, &set);
  if (r) return r;
  r = run_blob(h, ba, *set, s);
  if (r) return r;
  return note_uses(h, set, false, s, &h->blob_users);
}

extern "C" int32_t trik_hsv_blob_preview(TRIK_VIDTRANSCODE_CV_Handle h, const TrikHsvFrameBatch* b,
                                         const uint8_t* meta, const int32_t* top, int32_t out_width,
                                         int32_t out_height, int32_t out_line_length, uint8_t* previews,
                                         int64_t preview_stride, void* stream) {
  if (!h) return fail(TRIK_IVIDTRANSCODE_EFAIL, "handle is NULL");
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (b->layout != TRIK_HSV_LAYOUT_OV7670)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "the multi-blob sensor takes the ov7670 layout (YUV422P)");
  if (out_width < 0 || out_height < 0 || out_line_length < 2 * out_width)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "preview geometry: need out_line_length >= 2*out_width");
  const int64_t pb = (int64_t)out_height * out_line_length;
  if (b->n_frames > 1 && preview_stride < pb)
    return fail(TRIK_IVIDTRANSCODE_EFAIL, "preview_stride smaller than one preview");
  if (b->n_frames > 0 && pb > 0 && (!previews || !meta || !top)) return fail(TRIK_IVIDTRANSCODE_EFAIL, "NULL buffer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  std::lock_guard<std::mutex> lock(h->mu);
  DeviceGuard dg(h->device);
  if (b->n_frames == 0 || pb == 0) return 0;
  int32_t rc = check_device(h, b, previews);
  if (rc) return rc;
  rc = ensure_maps(h, b->width, b->height, out_width, out_height, s);
  if (rc) return rc;
  TRIK_VIDTRANSCODE_CV_InArgsAlg none;
  memset(&none, 0, sizeof none);
  PreviewArgs pa = preview_args(h, *b, none, out_width, out_height, out_line_length, previews, preview_stride);
  pa.meta = meta;
  HIP_TRY(launch_preview_body(pa, s));
  HIP_TRY(launch_blob_overlay(pa, top, s));
  return note_uses(h, nullptr, true, s);
}

extern "C" int32_t trik_hsv_synth(const TrikHsvFrameBatch* b, int32_t first_frame, int32_t kind,
                                  uint64_t seed, void* stream) {
  const std::string e = validate_batch(b);
  if (!e.empty()) return fail(TRIK_IVIDTRANSCODE_EFAIL, e);
  if (kind != 0 && kind != 1) return fail(TRIK_IVIDTRANSCODE_EFAIL, "kind must be 0 or 1");
  HIP_TRY(launch_synth(*b, const_cast<uint8_t*>(static_cast<const uint8_t*>(b->frames)), first_frame,
                       kind, seed, static_cast<hipStream_t>(stream)));
  return 0;
}
