// trik_hsv_group.cpp -- the multi-GPU layer of the C ABI.
//
// Frames are independent units, so a batch is sharded by frame index: each
// GPU processes its shard resident in its own HBM and the one exchange is the
// sum of the per-target batch totals (n_ranges x 3 int64) -- one RCCL
// all-reduce over xGMI, latency-bound, so no bucketing.  Two shapes:
//
//  * a group: one process drives several GPUs -- per device an object-sensor
//    handle, a HIP stream and a persistent host worker thread that enqueues
//    that device's work; an RCCL communicator over the devices
//    (ncclCommInitAll);
//  * a comm: one process per GPU (the torch.distributed / bench.py layout) --
//    an RCCL communicator over the ranks (ncclCommInitRank) for the totals.
//
// The reference has no multi-device path (one DSP, one frame per process
// call: trik/webcam/object_sensor/src/vidtranscode_cv_fxns.c:174-264); this
// extends its batched surface.  RCCL is loaded with dlopen on first use, so
// the library itself does not depend on it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "trik_hsv_internal.h"

using trik_hsv::set_error;

namespace {

// ---------------------------------------------------------------------------
// RCCL, resolved at run time
// ---------------------------------------------------------------------------
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string error;  // why loading failed ("" when loaded)
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* so = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((so = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!so) {
      const char* e = dlerror();
      r.error = std::string("cannot load librccl: ") + (e ? e : "not found");
      return;
    }
    auto sym = [&](const char* name, auto& f) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(so, name));
      if (!f && r.error.empty()) r.error = std::string("librccl lacks ") + name;
    };
    sym("ncclGetUniqueId", r.get_unique_id);
    sym("ncclCommInitRank", r.comm_init_rank);
    sym("ncclCommInitAll", r.comm_init_all);
    sym("ncclAllReduce", r.all_reduce);
    sym("ncclCommDestroy", r.comm_destroy);
    sym("ncclCommAbort", r.comm_abort);
    sym("ncclGroupStart", r.group_start);
    sym("ncclGroupEnd", r.group_end);
    sym("ncclGetErrorString", r.error_string);
  });
  return r;
}

int32_t nccl_fail(const char* what, ncclResult_t e) {
  return set_error(TRIK_IVIDTRANSCODE_EFAIL,
                   std::string(what) + ": " + (rccl().error_string ? rccl().error_string(e) : "RCCL error"));
}

int32_t need_rccl() {
  const Rccl& r = rccl();
  return r.error.empty() ? 0 : set_error(TRIK_IVIDTRANSCODE_EFAIL, r.error);
}

// ---------------------------------------------------------------------------
// A persistent host thread per device: runs one job at a time
// ---------------------------------------------------------------------------
class Worker {
 public:
  Worker() : th_([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  // Starts job on the worker; wait() returns its result and error message.
  void post(std::function<int32_t()> job) {
    std::lock_guard<std::mutex> l(mu_);
    job_ = std::move(job);
    busy_ = true;
    cv_.notify_all();
  }
  int32_t wait(std::string* err) {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [this] { return !busy_; });
    *err = err_;
    return rc_;
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> l(mu_);
    for (;;) {
      cv_.wait(l, [this] { return stop_ || (busy_ && job_); });
      if (stop_) return;
      std::function<int32_t()> job = std::move(job_);
      job_ = nullptr;
      l.unlock();
      const int32_t rc = job();
      const std::string err = rc ? std::string(trik_hsv_last_error()) : std::string();
      l.lock();
      rc_ = rc;
      err_ = err;
      busy_ = false;
      cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::function<int32_t()> job_;
  bool busy_ = false, stop_ = false;
  int32_t rc_ = 0;
  std::string err_;
  std::thread th_;  // last: starts after the members it uses
};

}  // namespace

struct TrikHsvGroup {
  std::vector<int> devices;
  std::vector<TRIK_VIDTRANSCODE_CV_Handle> handles;
  std::vector<hipStream_t> streams;
  std::vector<ncclComm_t> comms;
  std::vector<std::unique_ptr<Worker>> workers;
  std::mutex mu;  // one group call at a time
  // a collective failed to enqueue on some device: the communicators were
  // aborted (peers that had enqueued theirs do not wait forever) and the
  // group only accepts trik_hsv_group_delete (and _sync) from then on
  bool broken = false;

  // Runs job(d) on every device's worker (its device current) and waits;
  // the first failure is reported on the calling thread.
  int32_t each(const std::function<int32_t(int)>& job) {
    for (size_t d = 0; d < workers.size(); ++d) {
      const int dev = devices[d];
      workers[d]->post([&job, d, dev]() -> int32_t {
        if (hipSetDevice(dev) != hipSuccess)
          return set_error(TRIK_IVIDTRANSCODE_EFAIL, "hipSetDevice(" + std::to_string(dev) + ") failed");
        return job((int)d);
      });
    }
    int32_t rc = 0;
    std::string first;
    for (size_t d = 0; d < workers.size(); ++d) {
      std::string err;
      const int32_t r = workers[d]->wait(&err);
      if (r && !rc) {
        rc = r;
        first = "device " + std::to_string(devices[d]) + ": " + err;
      }
    }
    return rc ? set_error(rc, first) : 0;
  }

  // Aborts every communicator: RCCL kernels already enqueued return, so the
  // streams drain.
  void abort_comms() {
    for (size_t d = 0; d < comms.size(); ++d)
      if (comms[d]) {
        (void)hipSetDevice(devices[d]);
        (void)rccl().comm_abort(comms[d]);
        comms[d] = nullptr;
      }
    broken = true;
  }

  void release() {
    for (size_t d = 0; d < devices.size(); ++d) {
      (void)hipSetDevice(devices[d]);
      if (d < streams.size() && streams[d]) (void)hipStreamSynchronize(streams[d]);
      if (d < comms.size() && comms[d]) (void)rccl().comm_destroy(comms[d]);
      if (d < handles.size() && handles[d]) (void)TRIK_VIDTRANSCODE_CV_delete(handles[d]);
      if (d < streams.size() && streams[d]) (void)hipStreamDestroy(streams[d]);
    }
    workers.clear();  // joins the threads
  }
};

struct TrikHsvComm {
  ncclComm_t comm = nullptr;
  int device = 0;
};

extern "C" int32_t trik_hsv_group_create(int32_t n, const int32_t* devices, TRIK_HSV_GroupHandle* out) {
  if (!out) return set_error(TRIK_IALG_EFAIL, "out_group is NULL");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
  if (n < 1 || !devices) return set_error(TRIK_IALG_EFAIL, "group_create: need n_devices >= 1 and a device list");
  for (int i = 0; i < n; ++i) {
    if (devices[i] < 0 || devices[i] >= count)
      return set_error(TRIK_IALG_EFAIL, "group_create: no HIP device " + std::to_string(devices[i]));
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i])
        return set_error(TRIK_IALG_EFAIL, "group_create: device " + std::to_string(devices[i]) + " listed twice");
  }
  if (int32_t rc = need_rccl()) return rc;
  int prev = 0;
  (void)hipGetDevice(&prev);
  auto g = std::make_unique<TrikHsvGroup>();
  g->devices.assign(devices, devices + n);
  g->handles.assign(n, nullptr);
  g->streams.assign(n, nullptr);
  g->comms.assign(n, nullptr);
  int32_t rc = 0;
  for (int d = 0; d < n && !rc; ++d) {
    if (hipSetDevice(devices[d]) != hipSuccess || hipStreamCreateWithFlags(&g->streams[d], hipStreamNonBlocking) != hipSuccess)
      rc = set_error(TRIK_IALG_EFAIL, "group_create: stream on device " + std::to_string(devices[d]));
    else
      rc = TRIK_VIDTRANSCODE_CV_create(nullptr, &g->handles[d]);  // binds to devices[d]
  }
  if (!rc) {
    const ncclResult_t e = rccl().comm_init_all(g->comms.data(), n, g->devices.data());
    if (e != ncclSuccess) rc = nccl_fail("ncclCommInitAll", e);
  }
  if (!rc)
    for (int d = 0; d < n; ++d) g->workers.push_back(std::make_unique<Worker>());
  (void)hipSetDevice(prev);
  if (rc) {
    g->release();
    return rc;
  }
  *out = g.release();
  return TRIK_IALG_EOK;
}

extern "C" int32_t trik_hsv_group_process(TRIK_HSV_GroupHandle g, const TrikHsvFrameBatch* batches,
                                          const TRIK_VIDTRANSCODE_CV_InArgsAlg* ranges, int32_t n,
                                          TrikHsvTargetSums* const* sums, TrikHsvTarget* const* targets,
                                          TrikHsvTargetSums* const* totals) {
  if (!g || !batches || !sums || !totals) return set_error(TRIK_IVIDTRANSCODE_EFAIL, "group_process: NULL argument");
  if (n < 1 || n > TRIK_HSV_MAX_RANGES || !ranges)
    return set_error(TRIK_IVIDTRANSCODE_EFAIL, "n_ranges must be 1..64");
  for (size_t d = 0; d < g->devices.size(); ++d)
    if (!totals[d]) return set_error(TRIK_IVIDTRANSCODE_EFAIL, "group_process: totals_dev[" + std::to_string(d) + "] is NULL");
  std::lock_guard<std::mutex> lock(g->mu);
  if (g->broken) return set_error(TRIK_IVIDTRANSCODE_EFAIL, "group_process: a collective failed earlier; delete the group");
  // 1. every device, on its worker thread: its shard, then the totals of its
  //    frames (all enqueued before any collective: a failure here returns
  //    before any device has an all-reduce waiting for its peers)
  int32_t rc = g->each([&](int d) -> int32_t {
    const TrikHsvFrameBatch& b = batches[d];
    hipStream_t s = g->streams[d];
    if (b.n_frames > 0)  // the full step: one launch per 4 ranges where the fused step applies
      return trik_hsv_process_batch_totals(g->handles[d], &b, ranges, n, sums[d], targets ? targets[d] : nullptr,
                                           totals[d], s);
    return trik_hsv_batch_totals(0, n, sums[d], totals[d], s);
  });
  if (rc) return rc;
  // 2. one all-reduce of n x 3 int64 over the devices, issued from this
  //    thread as one RCCL group (the single-process multi-device pattern:
  //    every device's part is enqueued together or the group fails).  If it
  //    fails, the communicators are aborted so that no device's part waits
  //    for a peer that never joined, and the group is marked broken.
  int prev = 0;
  (void)hipGetDevice(&prev);
  ncclResult_t e = rccl().group_start();
  const char* what = "ncclGroupStart";
  const bool started = e == ncclSuccess;
  for (size_t d = 0; e == ncclSuccess && d < g->devices.size(); ++d) {
    e = rccl().all_reduce(totals[d], totals[d], (size_t)3 * n, ncclInt64, ncclSum, g->comms[d], g->streams[d]);
    what = "ncclAllReduce";
  }
  if (started) {  // a started group is always ended
    const ncclResult_t e2 = rccl().group_end();
    if (e == ncclSuccess && e2 != ncclSuccess) {
      e = e2;
      what = "ncclGroupEnd";
    }
  }
  (void)hipSetDevice(prev);
  if (e == ncclSuccess) return 0;
  g->abort_comms();
  return nccl_fail(what, e);
}

extern "C" int32_t trik_hsv_group_sync(TRIK_HSV_GroupHandle g) {
  if (!g) return set_error(TRIK_IVIDTRANSCODE_EFAIL, "group is NULL");
  std::lock_guard<std::mutex> lock(g->mu);
  // (after a failed collective the aborted communicators' kernels have
  // returned, so this does not block on them)
  return g->each([&](int d) -> int32_t {
    const hipError_t e = hipStreamSynchronize(g->streams[d]);
    return e == hipSuccess ? 0 : set_error(TRIK_IVIDTRANSCODE_EFAIL, std::string("hipStreamSynchronize: ") + hipGetErrorString(e));
  });
}

extern "C" void* trik_hsv_group_stream(TRIK_HSV_GroupHandle g, int32_t d) {
  if (!g || d < 0 || d >= (int32_t)g->streams.size()) return nullptr;
  return g->streams[d];
}

extern "C" int32_t trik_hsv_group_delete(TRIK_HSV_GroupHandle g) {
  if (!g) return set_error(TRIK_IALG_EFAIL, "group is NULL");
  int prev = 0;
  (void)hipGetDevice(&prev);
  g->release();
  delete g;
  (void)hipSetDevice(prev);
  return TRIK_IALG_EOK;
}

extern "C" int32_t trik_hsv_comm_id(uint8_t id[TRIK_HSV_COMM_ID_BYTES]) {
  static_assert(TRIK_HSV_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "comm id size");
  if (!id) return set_error(TRIK_IALG_EFAIL, "id is NULL");
  if (int32_t rc = need_rccl()) return rc;
  ncclUniqueId u;
  const ncclResult_t e = rccl().get_unique_id(&u);
  if (e != ncclSuccess) return nccl_fail("ncclGetUniqueId", e);
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return TRIK_IALG_EOK;
}

extern "C" int32_t trik_hsv_comm_create(int32_t n_ranks, int32_t rank, const uint8_t id[TRIK_HSV_COMM_ID_BYTES],
                                        TRIK_HSV_CommHandle* out) {
  if (!out || !id) return set_error(TRIK_IALG_EFAIL, "comm_create: NULL argument");
  *out = nullptr;
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return set_error(TRIK_IALG_EFAIL, "comm_create: bad rank");
  if (int32_t rc = need_rccl()) return rc;
  auto c = std::make_unique<TrikHsvComm>();
  if (hipGetDevice(&c->device) != hipSuccess) return set_error(TRIK_IALG_EFAIL, "no HIP device");
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  const ncclResult_t e = rccl().comm_init_rank(&c->comm, n_ranks, u, rank);
  if (e != ncclSuccess) return nccl_fail("ncclCommInitRank", e);
  *out = c.release();
  return TRIK_IALG_EOK;
}

extern "C" int32_t trik_hsv_comm_all_reduce_totals(TRIK_HSV_CommHandle c, TrikHsvTargetSums* totals, int32_t n,
                                                   void* stream) {
  if (!c || !totals) return set_error(TRIK_IVIDTRANSCODE_EFAIL, "comm_all_reduce_totals: NULL argument");
  if (n < 1 || n > TRIK_HSV_MAX_RANGES) return set_error(TRIK_IVIDTRANSCODE_EFAIL, "n_ranges must be 1..64");
  const ncclResult_t e =
      rccl().all_reduce(totals, totals, (size_t)3 * n, ncclInt64, ncclSum, c->comm, static_cast<hipStream_t>(stream));
  return e == ncclSuccess ? 0 : nccl_fail("ncclAllReduce", e);
}

extern "C" int32_t trik_hsv_comm_delete(TRIK_HSV_CommHandle c) {
  if (!c) return set_error(TRIK_IALG_EFAIL, "comm is NULL");
  if (c->comm) (void)rccl().comm_destroy(c->comm);
  delete c;
  return TRIK_IALG_EOK;
}
