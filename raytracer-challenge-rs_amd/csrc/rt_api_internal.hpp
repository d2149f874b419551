// rt_api_internal.hpp — what the C-ABI's translation units share (internal to
// librtamd.so, hidden visibility; not part of include/rt_render.h):
//   rt_api.cpp        errors, ABI sizes, pinned host buffers, camera / matrix, dev hooks
//   rt_scene.cpp      rt_scene_create*: flattening, hierarchies, upload
//   rt_workspace.cpp  the workspace pool's render call (run_render), overflow checks,
//                     device-to-host copies
//   rt_render.cpp     the render entry points (device shards, batches, host canvas,
//                     PPM, ray batches)
//   rt_multi.cpp      rt_render_multi and the RCCL hooks
//
// Product code: no CPU fallback anywhere. Every render entry point runs the
// HIP kernels (rt_wavefront.hip, rt_kernels.hip) and fails loudly
// (RT_ERR_HIP / RT_ERR_NO_DEVICE) when no device is usable.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_render.h"
#include "host/rt_math.hpp"
#include "rt_bvh.hpp"
#include "rt_kernels.hpp"
#include "rt_layout.hpp"
#include "rt_ppm_dev.hpp"
#include "rt_wavefront.hpp"

using namespace rtamd;

namespace rtapi __attribute__((visibility("hidden"))) {

extern thread_local std::string g_err;  // rt_last_error's text (rt_api.cpp)
// scene-creation knobs (rtamd_tuning_set, rt_api.cpp):
extern int g_bvh_leaf;  // BVH leaf size; 0 = automatic: 2, or 1 when the LDS image cannot hold the scene
extern int g_bvh_ct;    // SAH node-visit cost in percent of a sphere test
extern int g_lb_res;    // light-buffer cells per cube-map face edge: 0 = none, -1 = by scene size
// render-time tuning copied into every scene at its creation (rt_scene::tune)
extern std::mutex g_tune_mu;
extern WfTuning g_tune_defaults;

// `p .. p+n` lies in one pinned block of rt_host_buffer_alloc's pool (rt_api.cpp)
bool pinned_block(const void* p, size_t n);

inline int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// Nothing may throw across the C ABI (the Rust side maps codes to
// errors, an unwinding C++ exception would abort the caller): every int entry
// point runs its body through guarded().
template <typename F>
int guarded(F&& body) noexcept {
  try {
    return body();
  } catch (const std::bad_alloc&) {
    g_err = "out of memory";  // short: no allocation
    return RT_ERR_HOST;
  } catch (const std::exception& e) {
    try { g_err = e.what(); } catch (...) { g_err.clear(); }
    return RT_ERR_HOST;
  } catch (...) {
    g_err = "host error";
    return RT_ERR_HOST;
  }
}

// The caller's current device survives every entry point (SURVEY §8b:
// callable from any host thread; a multi-device caller's own choice of device
// must not change under it): an entry point that selects the scene's device
// holds a DeviceGuard, which restores the previous device on every return.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) {
      prev = -1;
      (void)hipGetLastError();
    }
  }
  explicit DeviceGuard(int dev) : DeviceGuard() { err = hipSetDevice(dev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

}  // namespace rtapi

#define RT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess)                                                              \
      return rtapi::fail(RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define RT_DEVICE(dev)                                                                             \
  rtapi::DeviceGuard _dev_guard(dev);                                                              \
  if (_dev_guard.err != hipSuccess)                                                                \
    return rtapi::fail(RT_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(_dev_guard.err))

constexpr int kMaxBands = 4;  // rt_render's row bands (WfTuning::bands, render_banded; more were slower: a stream each)

struct rt_scene {
  int device = 0;
  DevScene dev{};
  // device allocations
  void* d_blob = nullptr;       // trace + shade + light records
  hipStream_t stream = nullptr;  // rt_render_multi's stream on this device
  // Host-buffer entry points (rt_render*, rt_render_ppm, the batch calls) run
  // in a context of their own, taken from this pool for the call: a private
  // stream, device buffers for the input and output, and the pinned chunks of
  // the device-to-host copy. The scene's lock is held only while a call takes
  // or returns a context and while it enqueues work; its waits on the device
  // and its copies to the host run unlocked, so threads rendering one scene
  // overlap (each on its own stream and workspace).
  struct HostCtx {
    hipStream_t stream = nullptr;
    double* d_out = nullptr;  // output (doubles)
    size_t out_cap = 0;
    double* d_in = nullptr;   // batch input
    size_t in_cap = 0;
    char* d_ppm = nullptr;    // rt_render_ppm: the text and its row lengths / offsets
    size_t ppm_cap = 0;
    void* d_ppm_rows = nullptr;
    size_t ppm_rows_cap = 0;  // rows
    void* h_stage[2] = {nullptr, nullptr};  // device-to-host copies into caller memory: two pinned chunks
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    // banded host renders (render_banded): a stream per band after the first, and the
    // events that start each band when the previous band's render is done
    hipStream_t band_stream[kMaxBands - 1] = {};
    hipEvent_t band_ev[kMaxBands] = {};
    unsigned long long* h_len = nullptr;  // rt_render_ppm: the text's length (a pinned word)
    bool busy = false;
  };
  std::deque<HostCtx> ctxs;  // deque: a context's address survives the pool's growth
  std::mutex mu;  // the workspace and context pools, tuning, sizing (held only to enqueue)
  // Wavefront workspaces (queues grow on demand), one per stream in use, at
  // most kMaxWorkspaces unpinned: renders issued on different streams run
  // concurrently on the device (frames in flight). A workspace
  // taken over by another stream is reused in stream order: the new stream
  // first waits on the event recorded after the workspace's last render. A
  // synchronous call pins its workspace until it has read it back (its
  // counters, its overflow record), so no other stream takes it over meanwhile.
  struct WfSlot {
    std::unique_ptr<Wavefront> wf;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    unsigned long long tick = 0;
    int pins = 0;
  };
  // (16: a caller with 4 render streams, rt_render's 4 band streams, its own context
  // stream and a current stream stays below it, so no workspace is taken over by a
  // stream whose frames need larger arenas: a takeover that regrows them frees and
  // reallocates device memory, which synchronises the device)
  static constexpr size_t kMaxWorkspaces = 16;
  std::deque<WfSlot> wfs;
  unsigned long long tick = 0;
  WfSlot* last_wf = nullptr;
  bool prof_on = false;
  // rt_render_multi's communicators and buffers, cached on scenes[0]
  struct MultiCache {
    std::vector<rt_scene*> scenes;
    std::vector<ncclComm_t> comms;
    std::vector<double*> send;
    std::vector<size_t> send_cap;
    double* recv = nullptr;  // on device 0
    size_t recv_cap = 0;
    std::vector<hipEvent_t> ev0, ev1;  // per device: around its shard render (stats->ms_kernel)
    void release() {
      for (size_t i = 0; i < send.size(); ++i) {
        (void)hipSetDevice((int)i);
        if (send[i]) (void)hipFree(send[i]);
        if (i < comms.size() && comms[i]) (void)ncclCommDestroy(comms[i]);
        if (i < ev0.size() && ev0[i]) (void)hipEventDestroy(ev0[i]);
        if (i < ev1.size() && ev1[i]) (void)hipEventDestroy(ev1[i]);
      }
      (void)hipSetDevice(0);
      if (recv) (void)hipFree(recv);
      *this = MultiCache{};
    }
  } multi;
  std::mutex multi_mu;
  int prof_mask = (1 << WF_NCLASS) - 1;
  int n_objects = 0, n_lights = 0;
  WfTuning tune;  // this scene's render-time tuning (read under `mu` by every render)
  WfSizing sizing;  // the fast path's queue arenas, learned from this scene's frames (under `mu`)
  // ... and from the row bands of rt_render (render_banded): a band's rays per root ray
  // differ from a whole frame's (a band of floor reflects more than the frame), and
  // must not resize the arenas of whole-frame renders (a regrowth reallocates them)
  WfSizing band_sizing;
  ~rt_scene() {
    for (WfSlot& w : wfs)
      if (w.done) (void)hipEventDestroy(w.done);
    for (HostCtx& c : ctxs) {
      if (c.stream) {
        (void)hipStreamSynchronize(c.stream);
        (void)hipStreamDestroy(c.stream);
      }
      (void)hipFree(c.d_out); (void)hipFree(c.d_in); (void)hipFree(c.d_ppm); (void)hipFree(c.d_ppm_rows);
      for (int k = 0; k < 2; ++k) {
        if (c.h_stage[k]) (void)hipHostFree(c.h_stage[k]);
        if (c.stage_ev[k]) (void)hipEventDestroy(c.stage_ev[k]);
      }
      for (hipStream_t bs : c.band_stream)
        if (bs) {
          (void)hipStreamSynchronize(bs);
          (void)hipStreamDestroy(bs);
        }
      for (hipEvent_t be : c.band_ev)
        if (be) (void)hipEventDestroy(be);
      if (c.h_len) (void)hipHostFree(c.h_len);
    }
  }
  // A host context for one call (under `mu`); returned by release_ctx.
  hipError_t take_ctx(HostCtx** out) {
    for (HostCtx& c : ctxs)
      if (!c.busy) {
        c.busy = true;
        *out = &c;
        return hipSuccess;
      }
    ctxs.emplace_back();
    HostCtx& c = ctxs.back();
    const hipError_t e = hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      ctxs.pop_back();
      return e;
    }
    c.busy = true;
    *out = &c;
    return hipSuccess;
  }
  // the workspace for a render on `st` (stream-ordered after its previous user)
  hipError_t acquire(hipStream_t st, WfSlot** out) {
    WfSlot* pick = nullptr;
    // this stream's workspace, unless a synchronous call in flight holds it (pinned): two
    // calls on one stream must not share a workspace's counters and overflow record (the
    // call takes another workspace; stream order still runs the two renders in turn)
    for (WfSlot& w : wfs)
      if (w.stream == st && w.pins == 0) pick = &w;
    size_t unpinned = 0;
    for (WfSlot& w : wfs) unpinned += w.pins == 0;
    if (!pick && (wfs.size() < kMaxWorkspaces || unpinned == 0)) {
      wfs.emplace_back();
      pick = &wfs.back();
      pick->wf = std::make_unique<Wavefront>();
      hipError_t e = hipEventCreateWithFlags(&pick->done, hipEventDisableTiming);
      if (e != hipSuccess) return e;
      if (prof_on) pick->wf->set_profiling(true, prof_mask);
      pick->stream = st;
    }
    if (!pick) {  // take over the least recently used workspace that no call holds
      for (WfSlot& w : wfs)
        if (w.pins == 0 && (!pick || w.tick < pick->tick)) pick = &w;
      hipError_t e = hipStreamWaitEvent(st, pick->done, 0);
      if (e != hipSuccess) return e;
      pick->stream = st;
    }
    pick->tick = ++tick;
    last_wf = pick;
    *out = pick;
    return hipSuccess;
  }
};

namespace rtapi __attribute__((visibility("hidden"))) {

// ---- rt_workspace.cpp
int ensure_dev_buffer(double** buf, size_t* cap, size_t need);
// Device-to-host copy of n bytes into caller memory, stream-ordered after the
// work already on `st`; synchronous.
int copy_to_host(rt_scene::HostCtx* s, int d2h, void* dst, const void* src, size_t n, hipStream_t st);
int check_faults(rt_scene* s);
int run_render(rt_scene* s, const DevCamera& cam, const double* d_rays, uint32_t n_tasks, uint32_t aa,
               uint32_t max_depth, uint32_t row_block, uint32_t shard, uint32_t n_shards, double* d_out,
               hipStream_t stream, DevStats* stats_out = nullptr, float* ms_out = nullptr, uint32_t flags = 0,
               rt_scene::WfSlot** used = nullptr, const FrameTable* batch = nullptr, unsigned n_frames = 1,
               bool sync = false, std::unique_lock<std::mutex>* lk = nullptr, bool count = false,
               bool keep_pin = false, uint32_t blk_period = 0, uint64_t blk_mask = 0,
               hipEvent_t gen_ev = nullptr, int gen_ev_g = -1, bool* gen_ev_recorded = nullptr,
               WfSizing* sizing = nullptr);
void fill_stats(rt_stats* st, const DevStats& ds, float ms_kernel, double ms_total);
void add_stats(DevStats& sum, const DevStats& ds);

// ---- rt_render.cpp
// `Camera::render` into a host canvas in row bands, each band's copy behind the
// next bands' renders. `host_ready`: the canvas is already host-registered (or
// pinned) for the whole call. RT_ERR_NO_DEVICE: not bandable (render it whole).
int render_banded(rt_scene* s, std::unique_lock<std::mutex>& lk, rt_scene::HostCtx* c, const rt_camera_desc& cam,
                  uint32_t max_depth, uint32_t aa, double* out_rgb, bool host_ready = false);
// the fast path can serve `s` (a hierarchy to cull with, not switched off)
inline bool fast_path(const rt_scene* s) {
  return s->tune.accel != 0 && (s->dev.n_bvh > 0 || s->dev.n_obvh > 0 || s->dev.n_lbvh > 0);
}

inline PpmHeader ppm_header(uint32_t w, uint32_t h) {  // image/ppm.rs:53-63
  PpmHeader hd{};
  hd.n = (unsigned)std::snprintf(hd.s, sizeof hd.s, "P3\n%u %u\n255\n", w, h);
  return hd;
}

inline DevCamera to_dev_camera(const rt_camera_desc& c) {
  DevCamera d{};
  d.pixel_size = c.pixel_size;
  d.half_width = c.half_width;
  d.half_height = c.half_height;
  for (int i = 0; i < 12; ++i) d.inv[i] = c.inverse[i];
  d.hsize = c.hsize;
  d.vsize = c.vsize;
  return d;
}

inline bool valid_aa(uint32_t aa) { return aa == 1 || aa == 2 || aa == 4 || aa == 8 || aa == 16; }

inline bool valid_pattern(uint32_t period, uint64_t mask) {
  return period >= 1 && period <= 64 && mask != 0 && (period == 64 || (mask >> period) == 0);
}

// A host context for the duration of one entry point (rt_scene::HostCtx),
// returned to the pool under the scene's lock.
struct CtxLease {
  rt_scene* s;
  std::unique_lock<std::mutex>& lk;
  rt_scene::HostCtx* c = nullptr;
  ~CtxLease() {
    if (!c) return;
    if (!lk.owns_lock()) lk.lock();
    c->busy = false;
  }
};
#define RT_TAKE_CTX(lease)                                                           \
  do {                                                                               \
    const hipError_t _e = (lease).s->take_ctx(&(lease).c);                           \
    if (_e != hipSuccess) return rtapi::fail(RT_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(_e)); \
  } while (0)

}  // namespace rtapi
