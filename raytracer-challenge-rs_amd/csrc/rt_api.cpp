// rt_api.cpp — the C-ABI (include/rt_render.h): scene flattening/validation,
// device upload, render entry points, multi-GPU gather, PPM output.
//
// Product code: no CPU fallback anywhere. Every render entry point runs the
// HIP kernels (rt_wavefront.hip, rt_kernels.hip) and fails loudly
// (RT_ERR_HIP / RT_ERR_NO_DEVICE) when no device is usable.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <exception>
#include <functional>
#include <new>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
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

namespace {

thread_local std::string g_err;
int g_bvh_leaf = 0;     // BVH leaf size at scene creation (tuning knob "bvh_leaf"); 0 = automatic: 2, or 1 when
                        // the LDS image cannot hold the scene (C5: 1024² frame 4.42 -> 4.31 ms; C3 best at 2)
int g_bvh_ct = 70;      // SAH node-visit cost in percent of a sphere test (tuning knob "bvh_ct")
// light-buffer cells per cube-map face edge at scene creation ("lb_res"): 0 = none, -1 = by
// scene size (256, or 512 above 4096 diagonal spheres: C5 47.1 -> 46.7 ms/frame, C3 unchanged)
int g_lb_res = -1;
// render-time tuning copied into every scene at its creation (rt_scene::tune)
std::mutex g_tune_mu;
WfTuning g_tune_defaults;

// Pinned host buffers (rt_host_buffer_alloc): page-locked blocks the DMA
// engine writes at the full link rate, kept in a small pool on release so a
// frame loop's canvases reuse the same pages (no registration, no page faults).
// The pool is never torn down (the HIP runtime may be gone at process exit).
std::mutex g_pin_mu;
std::vector<std::pair<void*, size_t>> g_pin_live, g_pin_free;
size_t g_pin_free_bytes = 0;
constexpr size_t kPinPoolBytes = (size_t)1 << 30;

bool pinned_block(const void* p, size_t n) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  for (const auto& b : g_pin_live)
    if ((const char*)p >= (const char*)b.first && (const char*)p + n <= (const char*)b.first + b.second) return true;
  return false;
}

int fail(int code, const std::string& msg) {
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

#define RT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess)                                                              \
      return fail(RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(_e));      \
  } while (0)

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
#define RT_DEVICE(dev)                                                                             \
  DeviceGuard _dev_guard(dev);                                                                     \
  if (_dev_guard.err != hipSuccess)                                                                \
    return fail(RT_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(_dev_guard.err))

}  // namespace

// rt_last_error's text for entry points in other translation units (rt_ppm.cpp);
// internal to the library (hidden), not part of the ABI.
extern "C" __attribute__((visibility("hidden"))) int rtamd_fail(int code, const char* msg) noexcept {
  try {
    g_err = msg ? msg : "";
  } catch (...) {
    g_err.clear();
  }
  return code;
}

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

namespace {

bool is_diag_inverse(const double* inv) {
  return inv[1] == 0.0 && inv[2] == 0.0 && inv[4] == 0.0 && inv[6] == 0.0 && inv[8] == 0.0 &&
         inv[9] == 0.0;
}

bool m16_eq(const double* a, const double* b) {
  for (int i = 0; i < 16; ++i)
    if (!rt::equal(a[i], b[i])) return false;
  return true;
}
bool c3_eq(const double* a, const double* b) {
  return rt::equal(a[0], b[0]) && rt::equal(a[1], b[1]) && rt::equal(a[2], b[2]);
}

// Necessary condition for the reference's structural `Shape` equality
// (derived PartialEq of BaseShape, geometry/mod.rs:12; Material, material.rs:10;
// Pattern, pattern/mod.rs:17). The bounding box is left out, so this is a
// SUPERSET of the reference relation: "no pair passes" certifies that the
// containers walk never sees two structurally-equal objects.
bool may_be_equal(const rt_shape_desc& a, const rt_shape_desc& b) {
  if (a.kind != b.kind || (a.casts_shadow != 0) != (b.casts_shadow != 0)) return false;
  if (!m16_eq(a.transform, b.transform) || !m16_eq(a.inverse, b.inverse)) return false;
  if (!c3_eq(a.color, b.color)) return false;
  if (!(a.ambient == b.ambient && a.diffuse == b.diffuse && a.specular == b.specular &&
        a.shininess == b.shininess && a.reflective == b.reflective &&
        a.transparency == b.transparency && a.refractive_index == b.refractive_index))
    return false;
  if ((a.kind == RT_SHAPE_CYLINDER || a.kind == RT_SHAPE_CONE) &&
      !(a.minimum == b.minimum && a.maximum == b.maximum && (a.closed != 0) == (b.closed != 0)))
    return false;
  if (a.pattern_kind != b.pattern_kind) return false;
  if (a.pattern_kind != RT_PATTERN_NONE) {
    if (!m16_eq(a.pattern_transform, b.pattern_transform) ||
        !m16_eq(a.pattern_inverse, b.pattern_inverse))
      return false;
    if (a.pattern_kind != RT_PATTERN_TEST && !(c3_eq(a.pattern_a, b.pattern_a) && c3_eq(a.pattern_b, b.pattern_b)))
      return false;
  }
  return true;
}

int find_duplicate(const rt_shape_desc* s, size_t n, size_t* ia, size_t* ib) {
  std::vector<size_t> idx(n);
  for (size_t i = 0; i < n; ++i) idx[i] = i;
  // equal shapes have |translation-x difference| < EPSILON: sweep a sorted key
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return s[a].transform[3] < s[b].transform[3]; });
  for (size_t p = 0; p < n; ++p)
    for (size_t q = p + 1; q < n && s[idx[q]].transform[3] - s[idx[p]].transform[3] < rt::EPSILON; ++q)
      if (may_be_equal(s[idx[p]], s[idx[q]])) {
        *ia = std::min(idx[p], idx[q]);
        *ib = std::max(idx[p], idx[q]);
        return 1;
      }
  return 0;
}

int ensure_dev_buffer(double** buf, size_t* cap, size_t need) {
  if (*cap >= need) return RT_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  RT_HIP(hipMalloc(buf, std::max<size_t>(need, 1) * sizeof(double)));
  *cap = need;
  return RT_OK;
}

// Device-to-host copy of n bytes into caller (pageable) memory, stream-ordered
// after the work already on `st`: chunks land in two pinned buffers by DMA
// while the host copies the previous chunk out (a pageable hipMemcpy of a
// 50 MB canvas stages through the runtime at a few GB/s). Synchronous.
constexpr size_t kStageChunk = (size_t)8 << 20;
int copy_to_host(rt_scene::HostCtx* s, int d2h, void* dst, const void* src, size_t n, hipStream_t st) {
  if (n == 0) return RT_OK;
  if (pinned_block(dst, n)) {  // an rt_host_buffer_alloc block: the DMA engine writes it directly
    RT_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st));
    RT_HIP(hipStreamSynchronize(st));
    return RT_OK;
  }
  // Large copies: pin the caller's pages for this call and let the DMA engine
  // write them directly (one pass over the bytes instead of DMA + host memcpy).
  // The registration never outlives the call, so the caller may free or reuse
  // the buffer at once; a buffer that cannot be registered takes the chunks.
  if (n >= ((size_t)4 << 20) && d2h == 1) {
    if (hipHostRegister(dst, n, hipHostRegisterDefault) == hipSuccess) {
      hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      const hipError_t u = hipHostUnregister(dst);
      if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("device-to-host copy: ") + hipGetErrorString(e));
      // The frame is in dst and correct: a failed unregister is noted in
      // rt_last_error's text but does not discard it.
      if (u != hipSuccess) {
        (void)hipGetLastError();
        (void)fail(RT_OK, std::string("note: hipHostUnregister after a completed copy: ") + hipGetErrorString(u));
      }
      return RT_OK;
    }
    (void)hipGetLastError();  // not registrable (e.g. already pinned memory): the staging chunks below
  }
  for (int k = 0; k < 2; ++k) {
    if (!s->h_stage[k]) RT_HIP(hipHostMalloc(&s->h_stage[k], kStageChunk, hipHostMallocDefault));
    if (!s->stage_ev[k]) RT_HIP(hipEventCreateWithFlags(&s->stage_ev[k], hipEventDisableTiming));
  }
  const size_t n_chunks = (n + kStageChunk - 1) / kStageChunk;
  auto len = [&](size_t c) { return std::min(kStageChunk, n - c * kStageChunk); };
  // the host side of a chunk is copied out by a few threads (one thread's memcpy into
  // pageable memory runs well below the DMA rate)
  const unsigned n_threads = std::max(1u, std::min(4u, std::thread::hardware_concurrency() / 2));
  auto drain = [&](size_t c) -> int {
    RT_HIP(hipEventSynchronize(s->stage_ev[c & 1]));
    char* d = (char*)dst + c * kStageChunk;
    const char* src_h = (const char*)s->h_stage[c & 1];
    const size_t n_c = len(c);
    if (n_threads == 1 || n_c < ((size_t)1 << 20)) {
      std::memcpy(d, src_h, n_c);
      return RT_OK;
    }
    const size_t part = ((n_c + n_threads - 1) / n_threads + 4095) & ~(size_t)4095;
    std::vector<std::thread> pool;
    unsigned t = 1;
    try {  // nothing may throw across the C ABI: a thread that cannot start is copied here
      for (; t < n_threads && t * part < n_c; ++t)
        pool.emplace_back([=] { std::memcpy(d + t * part, src_h + t * part, std::min(part, n_c - t * part)); });
    } catch (...) {
    }
    for (unsigned u = t; u < n_threads && u * part < n_c; ++u)
      std::memcpy(d + u * part, src_h + u * part, std::min(part, n_c - u * part));
    std::memcpy(d, src_h, std::min(part, n_c));
    for (std::thread& th : pool) th.join();
    return RT_OK;
  };
  for (size_t c = 0; c < n_chunks; ++c) {
    if (c >= 2) {
      int rc = drain(c - 2);
      if (rc != RT_OK) return rc;
    }
    RT_HIP(hipMemcpyAsync(s->h_stage[c & 1], (const char*)src + c * kStageChunk, len(c), hipMemcpyDeviceToHost, st));
    RT_HIP(hipEventRecord(s->stage_ev[c & 1], st));
  }
  for (size_t c = n_chunks >= 2 ? n_chunks - 2 : 0; c < n_chunks; ++c) {
    int rc = drain(c);
    if (rc != RT_OK) return rc;
  }
  return RT_OK;
}

PpmHeader ppm_header(uint32_t w, uint32_t h) {  // image/ppm.rs:53-63
  PpmHeader hd{};
  hd.n = (unsigned)std::snprintf(hd.s, sizeof hd.s, "P3\n%u %u\n255\n", w, h);
  return hd;
}

DevCamera to_dev_camera(const rt_camera_desc& c) {
  DevCamera d{};
  d.pixel_size = c.pixel_size;
  d.half_width = c.half_width;
  d.half_height = c.half_height;
  for (int i = 0; i < 12; ++i) d.inv[i] = c.inverse[i];
  d.hsize = c.hsize;
  d.vsize = c.vsize;
  return d;
}

bool valid_aa(uint32_t aa) { return aa == 1 || aa == 2 || aa == 4 || aa == 8 || aa == 16; }

// A workspace whose fast-path frame overflowed its queue arenas (device-sized
// generations, Wavefront::take_overflow) fails the call that finds it: that
// earlier, asynchronous frame is incomplete. The arenas are grown past what
// the frame asked for, so the next frame fits at least that far.
int check_faults(rt_scene* s) {
  for (rt_scene::WfSlot& w : s->wfs) {
    if (w.pins || !w.wf->overflowed()) continue;  // a pinned workspace's own call handles its frame
    if (w.done) RT_HIP(hipEventSynchronize(w.done));  // its frames have run (the arenas are about to be reallocated)
    bool was = false;
    RT_HIP(w.wf->take_overflow(&was));
    if (was)
      return fail(RT_ERR_HIP, "wavefront queue arenas overflowed in an earlier asynchronous frame (that frame is "
                              "incomplete; the arenas have grown: render it again)");
  }
  return RT_OK;
}

// Launch one render (camera shard or ray batch) on `stream` through the
// wavefront pipeline. `n_tasks` root rays = pixels x aa (camera) or rays
// (batch). `stats_out`, when given, receives the exact counters and
// `ms_out` the kernel time. `sync`: the caller waits for this render anyway
// (a host canvas, the counters): the call waits for it, and a frame that
// overflowed its queue arenas is rendered again, with the arenas grown,
// until it fits (every synchronous entry point returns a complete frame).
// Asynchronous renders report an overflow later (check_faults). With `lk`
// (the scene's lock, held on entry and on return) the waits run unlocked;
// the workspace stays pinned to this call meanwhile. `used` receives the
// workspace; with `keep_pin` it stays pinned after the return (the caller
// reads it back and unpins it, under the scene's lock). `count`: the render
// counts the reference's rays (read_stats) without synchronising.
int run_render(rt_scene* s, const DevCamera& cam, const double* d_rays, uint32_t n_tasks, uint32_t aa,
               uint32_t max_depth, uint32_t row_block, uint32_t shard, uint32_t n_shards, double* d_out,
               hipStream_t stream, DevStats* stats_out = nullptr, float* ms_out = nullptr, uint32_t flags = 0,
               rt_scene::WfSlot** used = nullptr, const FrameTable* batch = nullptr, unsigned n_frames = 1,
               bool sync = false, std::unique_lock<std::mutex>* lk = nullptr, bool count = false,
               bool keep_pin = false, uint32_t blk_period = 0, uint64_t blk_mask = 0,
               hipEvent_t gen_ev = nullptr, int gen_ev_g = -1, bool* gen_ev_recorded = nullptr,
               WfSizing* sizing = nullptr) {
  WfSizing& sz = sizing ? *sizing : s->sizing;
  if (max_depth > (uint32_t)kMaxDepth)
    return fail(RT_ERR_INVALID_ARGUMENT, "max_depth > " + std::to_string(kMaxDepth));
  if (!valid_aa(aa)) return fail(RT_ERR_INVALID_ARGUMENT, "aa_samples must be 1, 2, 4, 8 or 16");
  if (flags & ~(uint32_t)RT_RENDER_EXHAUSTIVE) return fail(RT_ERR_INVALID_ARGUMENT, "unknown render flags");
  int rc = check_faults(s);
  if (rc != RT_OK) return rc;
  if (n_tasks == 0) {
    if (stats_out) *stats_out = DevStats{};
    if (ms_out) *ms_out = 0.f;
    if (used) *used = nullptr;
    return RT_OK;
  }
  rt_scene::WfSlot* w = nullptr;
  hipError_t e = s->acquire(stream, &w);
  if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("wavefront render: ") + hipGetErrorString(e));
  const unsigned wf_flags = ((flags & RT_RENDER_EXHAUSTIVE) ? WF_EXHAUSTIVE : 0u) |
                            ((count || stats_out) ? WF_COUNT : 0u) | (ms_out ? WF_TIME : 0u);
  sync = sync || stats_out || ms_out;
  struct Pin {  // the workspace is this call's until it returns (keep_pin: until the caller unpins it)
    rt_scene::WfSlot* w;
    bool on;
    ~Pin() {
      if (on) --w->pins;
    }
  } pin{w, sync && !keep_pin};
  if (sync || keep_pin) ++w->pins;
  if (keep_pin && used) *used = w;
  for (int attempt = 0;; ++attempt) {
    if (gen_ev) w->wf->set_gen_event(gen_ev, gen_ev_g);
    e = w->wf->render(s->dev, cam, d_rays == nullptr, d_rays, n_tasks, aa, max_depth, row_block, shard, n_shards,
                      d_out, stream, sz, nullptr, nullptr, s->tune, s->wfs.size() == 1, wf_flags, batch,
                      n_frames, blk_period, blk_mask);
    if (gen_ev) {
      if (gen_ev_recorded) *gen_ev_recorded = w->wf->gen_event_recorded();
      w->wf->set_gen_event(nullptr, -1);
    }
    if (e == hipSuccess) e = hipEventRecord(w->done, stream);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("wavefront render: ") + hipGetErrorString(e));
    if (!sync) break;
    if (lk) lk->unlock();
    e = hipStreamSynchronize(stream);
    if (lk) lk->lock();
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("wavefront render: ") + hipGetErrorString(e));
    w->wf->learn(sz);
    bool over = false;
    e = w->wf->take_overflow(&over);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("wavefront arenas: ") + hipGetErrorString(e));
    if (!over) break;
    if (attempt >= 24) return fail(RT_ERR_HIP, "wavefront queue arenas: the frame does not fit");
  }
  if (stats_out) RT_HIP(w->wf->read_stats(stats_out));
  if (ms_out) RT_HIP(w->wf->kernel_ms(ms_out));
  if (used) *used = w;
  return RT_OK;
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
    if (_e != hipSuccess) return fail(RT_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(_e)); \
  } while (0)

void fill_stats(rt_stats* st, const DevStats& ds, float ms_kernel, double ms_total) {
  std::memset(st, 0, sizeof *st);
  st->rays_shadow_traced = ds.rays_shadow_traced;
  st->sphere_tests_executed = ds.sphere_tests_executed;
  st->box_tests_executed = ds.box_tests_executed;
  st->exhaustive = ds.exhaustive;
  st->rays_primary = ds.rays_primary;
  st->rays_reflect = ds.rays_reflect;
  st->rays_refract = ds.rays_refract;
  st->rays_shadow = ds.rays_shadow;
  st->sphere_tests = ds.sphere_tests;
  st->plane_tests = ds.plane_tests;
  st->sphere_disc_ge0 = ds.sphere_disc_ge0;
  st->other_tests = ds.other_tests;
  st->ms_kernel = ms_kernel;
  st->ms_total = ms_total;
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }

// Development/benchmark hook (not in the public ABI): per-kernel-class timing
// of the wavefront pipeline. enable: 1 = on, 0 = off, -1 = just read. out[16]:
// ms[5] (primary, closest, shadow, prep, combine), rays[3], disc[3],
// n_diag, n_gen, n_planes, n_lights, n_quads, tests[3], boxes[3], bvh,
// n_bvh_nodes, bvh_depth, n_obvh_nodes, n_other_culled, lb_res, lb_items, sh_rays[2], sh_tests[2]
// (shadow rays / sphere tests inside the fused primary / secondary launches), fused,
// n_bvh_wide, wide_stack, n_lbvh_nodes, n_line_culled.
int rtamd_wf_profile(const rt_scene* cs, int enable, double out[38]) {
  if (!cs) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
  rt_scene* s = const_cast<rt_scene*>(cs);
  std::lock_guard<std::mutex> lk(s->mu);
  // enable: 0 off, 1 every kernel class, >= 2: (class mask << 1) | 1 (bench.py times one class)
  if (enable >= 0) {
    s->prof_on = enable != 0;
    s->prof_mask = enable > 1 ? (enable >> 1) : (1 << WF_NCLASS) - 1;
    for (rt_scene::WfSlot& w : s->wfs) w.wf->set_profiling(s->prof_on, s->prof_mask);
  }
  if (out) {
    RT_DEVICE(s->device);
    // class times: averaged over every frame profiled on any workspace; the
    // counters: the last frame
    WfProfile p{};
    double ms_sum[WF_NCLASS] = {};
    size_t frames = 0;
    for (rt_scene::WfSlot& w : s->wfs) {
      WfProfile q;
      RT_HIP(w.wf->last_profile(&q));
      const size_t f = w.wf->profiled_frames();
      for (int c = 0; c < WF_NCLASS; ++c) ms_sum[c] += q.ms[c] * (double)(f > 1 ? f : 1);
      frames += f > 1 ? f : (f == 1 ? 1 : 0);
      if (&w == s->last_wf) p = q;
    }
    for (int c = 0; c < WF_NCLASS; ++c) p.ms[c] = frames ? ms_sum[c] / (double)frames : 0.0;
    for (int i = 0; i < 5; ++i) out[i] = p.ms[i];
    for (int i = 0; i < 3; ++i) { out[5 + i] = p.rays[i]; out[8 + i] = p.disc[i]; }
    out[11] = s->dev.n_diag; out[12] = s->dev.n_gen; out[13] = s->dev.n_planes;
    out[14] = s->dev.n_lights; out[15] = s->dev.n_quads;
    for (int i = 0; i < 3; ++i) {
      out[16 + i] = p.bvh ? p.tests[i] : p.rays[i] * s->dev.n_diag;  // exhaustive: every ray tests every sphere
      out[19 + i] = p.boxes[i];
    }
    out[22] = p.bvh;
    out[23] = s->dev.n_bvh;
    out[24] = s->dev.bvh_depth;
    out[25] = s->dev.n_obvh;
    out[26] = s->dev.n_orec;
    out[27] = s->dev.lb_cells ? s->dev.lb_res : 0;
    out[28] = s->dev.lb_cells ? s->dev.lb_n_items : 0;
    for (int i = 0; i < 2; ++i) { out[29 + i] = p.sh_rays[i]; out[31 + i] = p.sh_tests[i]; }
    out[33] = p.fused;
    out[34] = s->dev.bvhw ? s->dev.n_bvhw : 0;
    out[35] = s->dev.bvhw ? s->dev.bvhw_stack : 0;
    out[36] = s->dev.n_lbvh;
    out[37] = s->dev.n_lrec;
  }
  return RT_OK;
}

// Development-only tuning hooks (not declared in include/rt_render.h).
// rtamd_tuning_set: the scene-creation knobs (lb_res, bvh_leaf, bvh_ct) and
// the render-time defaults copied into scenes created afterwards;
// rtamd_scene_tuning_set: one scene's render-time knobs (WfTuning).
int rtamd_tuning_set(const char* key, int value) {
  return guarded([&]() -> int {
  if (key && std::strcmp(key, "lb_res") == 0) {
    if (value < -1 || value > 512) return fail(RT_ERR_INVALID_ARGUMENT, "lb_res must be in [-1, 512]");
    g_lb_res = value;
    return RT_OK;
  }
  if (key && std::strcmp(key, "bvh_ct") == 0) {
    if (value < 1 || value > 10000) return fail(RT_ERR_INVALID_ARGUMENT, "bvh_ct must be in [1, 10000]");
    g_bvh_ct = value;
    return RT_OK;
  }
  if (key && std::strcmp(key, "bvh_leaf") == 0) {
    if (value < 0 || value > kBvhLeafMax) return fail(RT_ERR_INVALID_ARGUMENT, "bvh_leaf must be in [0, 127]");
    g_bvh_leaf = value;
    return RT_OK;
  }
  std::lock_guard<std::mutex> lk(g_tune_mu);
  const int r = wf_tuning_apply(g_tune_defaults, key, value);
  if (r < 0) return fail(RT_ERR_INVALID_ARGUMENT, std::string("bad value for tuning key ") + key);
  if (r == 0) return fail(RT_ERR_INVALID_ARGUMENT, "unknown tuning key");
  return RT_OK;
  });
}
int rtamd_scene_tuning_set(const rt_scene* scene, const char* key, int value) {
  return guarded([&]() -> int {
  if (!scene) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::lock_guard<std::mutex> lk(s->mu);
  const int r = wf_tuning_apply(s->tune, key, value);
  if (r < 0) return fail(RT_ERR_INVALID_ARGUMENT, std::string("bad value for tuning key ") + (key ? key : ""));
  if (r == 0) return fail(RT_ERR_INVALID_ARGUMENT, "unknown render-time tuning key (scene-creation keys: "
                                                   "rtamd_tuning_set before the scene is created)");
  return RT_OK;
  });
}
// Development hook (not in the public ABI): a non-blocking stream on the
// current device; cu_masked = 1 creates it through hipExtStreamCreateWithCUMask
// with every CU enabled (the runtime gives such a stream a hardware queue of
// its own instead of sharing one of the GPU_MAX_HW_QUEUES).
int rtamd_stream_create(int cu_masked, void** out) {
  if (!out) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  hipStream_t st = nullptr;
  if (cu_masked) {
    int dev = 0, n_cu = 0;
    RT_HIP(hipGetDevice(&dev));
    RT_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0xFFFFFFFFu);
    RT_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
  } else {
    RT_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  }
  *out = st;
  return RT_OK;
}
// Development/benchmark hooks (not in the public ABI): an RCCL communicator
// per render stream for multi-process frame assembly, so that a frame's
// gather is enqueued on the stream that rendered it (no cross-stream event;
// bench.py, rtamd.distributed.RcclStreamAssembler).
int rtamd_nccl_unique_id(unsigned char* out, size_t size) {
  if (!out || size < sizeof(ncclUniqueId)) return fail(RT_ERR_INVALID_ARGUMENT, "unique id buffer too small");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return fail(RT_ERR_RCCL, "ncclGetUniqueId");
  std::memcpy(out, &id, sizeof id);
  return RT_OK;
}
// The communicator is created non-blocking and waited for at most `timeout_ms`,
// so a rank whose peers failed before joining does not hang: it aborts the
// half-made communicator and returns RT_ERR_RCCL, and the caller's agreement
// step (RcclStreamAssembler) sends every rank to the fallback together.
namespace {
ncclResult_t nccl_wait(ncclComm_t c, ncclResult_t r, int timeout_ms) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (r == ncclInProgress) {
    if (std::chrono::steady_clock::now() > deadline) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    if (ncclCommGetAsyncError(c, &r) != ncclSuccess) return ncclInternalError;
  }
  return r;
}
}  // namespace
int rtamd_nccl_comm_init(int nranks, const unsigned char* id, size_t size, int rank, int device, int timeout_ms,
                         void** comm) {
  if (!id || !comm || size < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks || timeout_ms < 1)
    return fail(RT_ERR_INVALID_ARGUMENT, "bad communicator arguments");
  *comm = nullptr;
  RT_DEVICE(device);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  ncclComm_t c = nullptr;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&c, nranks, uid, rank, &cfg);
  if (c && (r == ncclSuccess || r == ncclInProgress)) r = nccl_wait(c, r, timeout_ms);
  if (r != ncclSuccess) {
    if (c) (void)ncclCommAbort(c);
    return fail(RT_ERR_RCCL, r == ncclInProgress ? "ncclCommInitRankConfig: timed out" : "ncclCommInitRankConfig");
  }
  *comm = c;
  return RT_OK;
}
int rtamd_nccl_gather_f64(const double* send, double* recv, size_t count, int root, void* comm, void* stream) {
  if (!send || !comm) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  ncclResult_t r = ncclGather(send, recv, count, ncclDouble, root, (ncclComm_t)comm, (hipStream_t)stream);
  // a non-blocking communicator may still be connecting: the enqueue completes in the background
  if (r == ncclInProgress) r = nccl_wait((ncclComm_t)comm, r, 120000);
  if (r != ncclSuccess) return fail(RT_ERR_RCCL, "ncclGather");
  return RT_OK;
}
int rtamd_nccl_comm_destroy(void* comm) {
  if (comm && ncclCommDestroy((ncclComm_t)comm) != ncclSuccess) return fail(RT_ERR_RCCL, "ncclCommDestroy");
  return RT_OK;
}
int rtamd_nccl_comm_abort(void* comm) {
  if (comm && ncclCommAbort((ncclComm_t)comm) != ncclSuccess) return fail(RT_ERR_RCCL, "ncclCommAbort");
  return RT_OK;
}
int rt_abi_version(void) { return RT_ABI_VERSION; }
size_t rt_sizeof_shape_desc(void) { return sizeof(rt_shape_desc); }
size_t rt_sizeof_camera_desc(void) { return sizeof(rt_camera_desc); }
size_t rt_sizeof_stats(void) { return sizeof(rt_stats); }
static_assert(sizeof(rt_shape_desc) == 680 && sizeof(rt_camera_desc) == 160 && sizeof(rt_stats) == 112,
              "ABI struct sizes (include/rt_render.h, INTEGRATION.md)");

void* rt_host_buffer_alloc(size_t bytes) {
  if (bytes == 0) {
    g_err = "rt_host_buffer_alloc: zero bytes";
    return nullptr;
  }
  try {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    for (size_t i = 0; i < g_pin_free.size(); ++i)
      if (g_pin_free[i].second >= bytes && g_pin_free[i].second <= bytes + bytes / 4) {  // a close fit
        const auto b = g_pin_free[i];
        g_pin_free.erase(g_pin_free.begin() + (long)i);
        g_pin_free_bytes -= b.second;
        g_pin_live.push_back(b);
        return b.first;
      }
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess || !p) {
      (void)hipGetLastError();
      g_err = "rt_host_buffer_alloc: hipHostMalloc failed";
      return nullptr;
    }
    g_pin_live.emplace_back(p, bytes);
    return p;
  } catch (...) {
    g_err = "out of memory";
    return nullptr;
  }
}

void rt_host_buffer_free(void* p) {
  if (!p) return;
  try {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    for (size_t i = 0; i < g_pin_live.size(); ++i)
      if (g_pin_live[i].first == p) {
        const auto b = g_pin_live[i];
        g_pin_live.erase(g_pin_live.begin() + (long)i);
        if (g_pin_free_bytes + b.second <= kPinPoolBytes) {
          g_pin_free.push_back(b);
          g_pin_free_bytes += b.second;
        } else {
          (void)hipHostFree(b.first);
        }
        return;
      }
  } catch (...) {
  }
}

int rt_scene_check(const rt_scene* scene) {
  return guarded([&]() -> int {
  if (!scene) return fail(RT_ERR_INVALID_ARGUMENT, "null scene");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::lock_guard<std::mutex> lk(s->mu);
  RT_DEVICE(s->device);
  for (rt_scene::WfSlot& w : s->wfs)
    if (w.done) RT_HIP(hipEventSynchronize(w.done));  // the workspace's last render (and its check) has run
  return check_faults(s);
  });
}

int rt_device_count(void) {
  return guarded([&]() -> int {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
  });
}

int rt_matrix_inverse(const double m[16], double out[16]) {
  return guarded([&]() -> int {
  if (!m || !out) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  rt::Matrix a = rt::Matrix::from_slice(4, 4, m);
  if (!a.is_invertible()) return fail(RT_ERR_NOT_INVERTIBLE, "matrix is not invertible (matrix.rs:139)");
  rt::Matrix inv = a.inverse();
  std::memcpy(out, inv.data(), 16 * sizeof(double));
  return RT_OK;
  });
}

// camera.rs:33-55 (+ set_transform :128-131)
int rt_camera_init(uint32_t hsize, uint32_t vsize, double field_of_view, const double transform[16],
                   rt_camera_desc* out) {
  return guarded([&]() -> int {
  if (!out || hsize == 0 || vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "bad camera size");
  const double half_view = std::tan(field_of_view / 2.0);
  const double aspect = (double)hsize / (double)vsize;
  double half_width, half_height;
  if (aspect >= 1.0) {
    half_width = half_view;
    half_height = half_view / aspect;
  } else {
    half_width = half_view * aspect;
    half_height = half_view;
  }
  out->hsize = hsize;
  out->vsize = vsize;
  out->pixel_size = half_width * 2.0 / (double)hsize;
  out->half_width = half_width;
  out->half_height = half_height;
  if (transform) {
    int rc = rt_matrix_inverse(transform, out->inverse);
    if (rc != RT_OK) return rc;
  } else {
    rt::Matrix id = rt::Matrix::identity(4, 4);
    std::memcpy(out->inverse, id.data(), sizeof out->inverse);
  }
  return RT_OK;
  });
}

int rt_scene_create(const rt_shape_desc* shapes, size_t n_shapes, const rt_light_desc* lights,
                    size_t n_lights, int device, rt_scene** out) {
  return guarded([&]() -> int {
  return rt_scene_create_groups(shapes, n_shapes, nullptr, nullptr, 0, lights, n_lights, device, out);
  });
}

int rt_scene_create_groups(const rt_shape_desc* shapes, size_t n_shapes, const int32_t* shape_group,
                           const rt_group_desc* groups, size_t n_groups, const rt_light_desc* lights,
                           size_t n_lights, int device, rt_scene** out) {
  return guarded([&]() -> int {
  if (!out || (n_shapes && !shapes) || (n_lights && !lights) || (n_groups && (!groups || !shape_group)))
    return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  *out = nullptr;
  if (n_shapes > (size_t)(1u << 29)) return fail(RT_ERR_INVALID_ARGUMENT, "too many shapes");
  if (n_groups > (size_t)(1u << 24)) return fail(RT_ERR_INVALID_ARGUMENT, "too many groups");
  for (size_t g = 0; g < n_groups; ++g)
    if (groups[g].parent < -1 || groups[g].parent >= (int32_t)g)
      return fail(RT_ERR_INVALID_ARGUMENT, "group " + std::to_string(g) + ": its parent must be -1 or an earlier group");
  // a shape's gate: 1 + its innermost group (0: none)
  auto gate_of = [&](size_t i) -> int32_t { return shape_group && n_groups ? shape_group[i] + 1 : 0; };
  for (size_t i = 0; i < n_shapes; ++i)
    if (gate_of(i) < 0 || gate_of(i) > (int32_t)n_groups)
      return fail(RT_ERR_INVALID_ARGUMENT, "shape " + std::to_string(i) + ": bad group index");
  for (size_t i = 0; i < n_shapes; ++i) {
    if (shapes[i].kind < RT_SHAPE_SPHERE || shapes[i].kind > RT_SHAPE_CONE)
      return fail(RT_ERR_UNSUPPORTED_SHAPE, "shape " + std::to_string(i) +
                                                ": supported kinds are Sphere, Plane, Cube, Cylinder, Cone");
    if (shapes[i].pattern_kind < RT_PATTERN_NONE || shapes[i].pattern_kind > RT_PATTERN_CHECKERS)
      return fail(RT_ERR_INVALID_ARGUMENT, "shape " + std::to_string(i) + ": bad pattern kind");
  }
  size_t da, db;
  if (find_duplicate(shapes, n_shapes, &da, &db))
    return fail(RT_ERR_DUPLICATE_SHAPES, "shapes " + std::to_string(da) + " and " + std::to_string(db) +
                                             " may be structurally equal (containers walk, intersection.rs:63-90)");

  int ndev = rt_device_count();
  if (ndev <= 0) return fail(RT_ERR_NO_DEVICE, "no HIP device available (no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID_ARGUMENT, "bad device ordinal");

  // ---- flatten (reference object order preserved through `meta`)
  std::vector<SphereDiag> diag;
  std::vector<SphereGen> gen;
  std::vector<PlaneRec> planes;
  std::vector<QuadRec> quads;
  std::vector<ShadeRec> shade(n_shapes);
  for (size_t i = 0; i < n_shapes; ++i) {
    const rt_shape_desc& d = shapes[i];
    const int64_t meta = ((int64_t)i << 1) | (d.casts_shadow ? 1 : 0);
    const int32_t gate = gate_of(i);  // shapes inside groups: general records with their group gate
    if (d.kind == RT_SHAPE_SPHERE) {
      if (is_diag_inverse(d.inverse) && gate == 0) {
        SphereDiag r{};
        r.s[0] = d.inverse[0]; r.s[1] = d.inverse[5]; r.s[2] = d.inverse[10];
        r.t[0] = d.inverse[3]; r.t[1] = d.inverse[7]; r.t[2] = d.inverse[11];
        r.meta = meta;
        diag.push_back(r);
      } else {
        SphereGen r{};
        for (int e = 0; e < 12; ++e) r.m[e] = d.inverse[e];
        r.meta = meta;
        r.gate = gate;
        gen.push_back(r);
      }
    } else if (d.kind == RT_SHAPE_PLANE) {
      PlaneRec r{};
      for (int e = 0; e < 4; ++e) r.m[e] = d.inverse[4 + e];
      r.meta = meta;
      r.gate = gate;
      planes.push_back(r);
    } else {
      QuadRec r{};
      for (int e = 0; e < 12; ++e) r.m[e] = d.inverse[e];
      r.minimum = d.minimum;
      r.maximum = d.maximum;
      r.kind = d.kind;
      r.closed = d.closed ? 1 : 0;
      r.meta = (int32_t)meta;
      r.gate = gate;
      quads.push_back(r);
    }
    ShadeRec& s = shade[i];
    std::memset(&s, 0, sizeof s);
    for (int e = 0; e < 12; ++e) s.inv[e] = d.inverse[e];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) s.invT[r * 3 + c] = d.inverse[c * 4 + r];  // transpose (matrix.rs:79-89)
    for (int c = 0; c < 3; ++c) s.color[c] = d.color[c];
    s.ambient = d.ambient; s.diffuse = d.diffuse; s.specular = d.specular; s.shininess = d.shininess;
    s.reflective = d.reflective; s.transparency = d.transparency; s.refractive_index = d.refractive_index;
    s.pattern_kind = d.pattern_kind;
    for (int c = 0; c < 3; ++c) { s.pat_a[c] = d.pattern_a[c]; s.pat_b[c] = d.pattern_b[c]; }
    for (int e = 0; e < 12; ++e) s.pat_inv[e] = d.pattern_inverse[e];
    s.kind = d.kind;
    s.shadow = d.casts_shadow ? 1 : 0;
    s.minimum = d.minimum;
    s.maximum = d.maximum;
  }
  // exact-culling hierarchy over the diagonal spheres (reorders `diag`; keys
  // come from `meta`, so the order changes no result)
  int bvh_depth = 0;
  const int leaf = g_bvh_leaf > 0 ? g_bvh_leaf : 2;
  std::vector<BvhNode> bvh = build_sphere_bvh(diag, leaf, &bvh_depth, g_bvh_ct / 100.0);
  if (g_bvh_leaf == 0 && !bvh.empty()) {
    // a scene whose pair image (stack, nodes, sphere records) does not fit in
    // LDS is traversed from global memory, where single-sphere leaves win
    const size_t image = (size_t)(bvh_depth + 1) * kFusedBlockThreads * 4 + bvh.size() * sizeof(BvhNode) +
                         diag.size() * sizeof(SphereDiag);
    if (image > kFusedLdsLimit) bvh = build_sphere_bvh(diag, 1, &bvh_depth, g_bvh_ct / 100.0);
  }
  const std::vector<BvhPair> bvh_pair = pair_layout(bvh);
  int wide_stack = 0;
  const std::vector<BvhWide> bvh_wide = wide_layout(bvh, diag, &wide_stack);
  const std::vector<BvhWide16> bvh_wide16 = wide16_layout(bvh_wide);
  // ... and over the other bounded records (general spheres, cubes, cylinders
  // with finite caps); the rest stays exhaustive on the fast path too
  std::vector<OtherRec> orec;
  std::vector<SphereGen> fx_gen;
  std::vector<QuadRec> fx_quads;
  double blo[3], bhi[3];
  // (shapes inside groups too: their group gate goes with them, tested before the
  // shape at the leaf, as the reference tests a group's box before its children)
  for (const SphereGen& g : gen) {
    OtherRec r{};
    for (int e = 0; e < 12; ++e) r.m[e] = g.m[e];
    r.kind = 0;
    r.meta = (int32_t)g.meta;
    r.gate = g.gate;
    if (other_box(r, blo, bhi)) orec.push_back(r);
    else fx_gen.push_back(g);
  }
  std::vector<QuadRec> line_rec;  // open tubes and cones with finite bounds: the line hierarchy
  for (const QuadRec& q : quads) {
    if (other_box(q, blo, bhi)) orec.push_back(q);
    else if (q.gate == 0 && line_box(q, blo, bhi)) line_rec.push_back(q);  // (grouped tubes and cones: exhaustive)
    else fx_quads.push_back(q);
  }
  std::vector<GroupRec> grec(n_groups);
  for (size_t g = 0; g < n_groups; ++g) {
    for (int c = 0; c < 3; ++c) { grec[g].lo[c] = groups[g].min[c]; grec[g].hi[c] = groups[g].max[c]; }
    grec[g].parent = groups[g].parent + 1;
  }
  // A handful of records is cheaper in the exhaustive loops (wave-uniform, scalar loads) than
  // behind a per-lane walk from global memory: the hierarchies start at kMinHierRecords
  // (640x480 frames: the groups scene's 7 grouped records 0.92 ms in the hierarchies, 0.69
  // exhaustive; solids 0.72 -> 0.60, zoo 0.37 -> 0.29; a divided group of 800: 5.1 against
  // 32.3), except in a scene without any other hierarchy, where one of
  // them is what opens the fused generations (the hexagon demo: 1.0 -> 0.53 ms)
  constexpr size_t kMinHierRecords = 16;
  int obvh_depth = 0;
  std::vector<BvhNode> obvh;
  if (orec.size() >= kMinHierRecords || (bvh.empty() && !orec.empty()))
    obvh = build_other_bvh(orec, leaf, &obvh_depth, g_bvh_ct / 100.0);
  if (obvh_depth > kBvhMaxDepth) obvh.clear();  // deeper than other_trace's stack: exhaustive
  int lbvh_depth = 0;
  std::vector<ConeCluster> lclus;
  std::vector<int32_t> lcone;
  std::vector<BvhNode> lbvh;
  if (line_rec.size() >= kMinHierRecords || (bvh.empty() && obvh.empty() && !line_rec.empty()))
    lbvh = build_line_bvh(line_rec, &lclus, &lcone, &lbvh_depth);
  if (lbvh.empty() || lbvh_depth > kBvhMaxDepth) {  // exhaustive, as before the line hierarchy
    for (const QuadRec& q : line_rec) fx_quads.push_back(q);
    line_rec.clear();
    lbvh.clear();
    lclus.clear();
    lcone.clear();
  }
  if (obvh.empty()) {  // (only when there are no records, or more than the leaf codes can index)
    for (const OtherRec& r : orec) {
      if (r.kind == 0) {
        SphereGen g{};
        for (int e = 0; e < 12; ++e) g.m[e] = r.m[e];
        g.meta = r.meta;
        g.gate = r.gate;
        fx_gen.push_back(g);
      } else {
        fx_quads.push_back(r);
      }
    }
    orec.clear();
  }
  std::vector<LightRec> lrec(n_lights);
  for (size_t i = 0; i < n_lights; ++i)
    for (int c = 0; c < 3; ++c) { lrec[i].pos[c] = lights[i].position[c]; lrec[i].intensity[c] = lights[i].intensity[c]; }
  // light buffers over the (reordered) diagonal spheres: the shadow rays' cell lists
  LightBuffer lb;
  const int lb_res = g_lb_res >= 0 ? g_lb_res : (diag.size() > 4096 ? 512 : 256);
  if (!diag.empty() && n_lights > 0 && n_lights <= (size_t)kLbMaxLights && lb_res > 0)
    lb = build_light_buffer(diag, lrec, lb_res);

  // ---- one blob, 64-B aligned sections
  auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_diag = 0;
  // one zeroed padding record after each trace section (look-ahead loads)
  const size_t o_gen = align(o_diag + (diag.size() + 1) * sizeof(SphereDiag));
  const size_t o_pl = align(o_gen + (gen.size() + 1) * sizeof(SphereGen));
  const size_t o_qd = align(o_pl + (planes.size() + 1) * sizeof(PlaneRec));
  const size_t o_bv = align(o_qd + (quads.size() + 1) * sizeof(QuadRec));
  const size_t o_bp = align(o_bv + (bvh.size() + 1) * sizeof(BvhNode));
  const size_t o_bw = align(o_bp + (bvh_pair.size() + 1) * sizeof(BvhPair));
  const size_t o_bh = align(o_bw + (bvh_wide.size() + 1) * sizeof(BvhWide));
  const size_t o_ob = align(o_bh + (bvh_wide16.size() + 1) * sizeof(BvhWide16));
  const size_t o_or = align(o_ob + (obvh.size() + 1) * sizeof(BvhNode));
  const size_t o_lb = align(o_or + (orec.size() + 1) * sizeof(OtherRec));
  const size_t o_lr = align(o_lb + (lbvh.size() + 1) * sizeof(BvhNode));
  const size_t o_cc = align(o_lr + (line_rec.size() + 1) * sizeof(QuadRec));
  const size_t o_lm = align(o_cc + (lclus.size() + 1) * sizeof(ConeCluster));
  const size_t o_fg = align(o_lm + (lcone.size() + 1) * sizeof(int32_t));
  const size_t o_fq = align(o_fg + (fx_gen.size() + 1) * sizeof(SphereGen));
  const size_t o_sh = align(o_fq + (fx_quads.size() + 1) * sizeof(QuadRec));
  const size_t o_rt = align(o_sh + shade.size() * sizeof(ShadeRec));
  const size_t o_li = align(o_rt + (shade.size() + 1) * 2 * sizeof(double));
  const size_t o_lc = align(o_li + lrec.size() * sizeof(LightRec));
  const size_t o_lv = align(o_lc + lb.cells.size() * sizeof(LbCell));
  const size_t o_ld = align(o_lv + (lb.ov.size() + 1) * sizeof(uint16_t));
  const size_t o_ll = align(o_ld + lb.delta.size() * sizeof(float));
  const size_t o_gr = align(o_ll + lb.limit.size() * sizeof(float));
  const size_t total = align(o_gr + grec.size() * sizeof(GroupRec)) + 256;
  std::vector<unsigned char> host(total, 0);
  if (!diag.empty()) std::memcpy(&host[o_diag], diag.data(), diag.size() * sizeof(SphereDiag));
  if (!gen.empty()) std::memcpy(&host[o_gen], gen.data(), gen.size() * sizeof(SphereGen));
  if (!planes.empty()) std::memcpy(&host[o_pl], planes.data(), planes.size() * sizeof(PlaneRec));
  if (!quads.empty()) std::memcpy(&host[o_qd], quads.data(), quads.size() * sizeof(QuadRec));
  if (!bvh.empty()) std::memcpy(&host[o_bv], bvh.data(), bvh.size() * sizeof(BvhNode));
  if (!bvh_pair.empty()) std::memcpy(&host[o_bp], bvh_pair.data(), bvh_pair.size() * sizeof(BvhPair));
  if (!bvh_wide.empty()) std::memcpy(&host[o_bw], bvh_wide.data(), bvh_wide.size() * sizeof(BvhWide));
  if (!bvh_wide16.empty()) std::memcpy(&host[o_bh], bvh_wide16.data(), bvh_wide16.size() * sizeof(BvhWide16));
  if (!obvh.empty()) std::memcpy(&host[o_ob], obvh.data(), obvh.size() * sizeof(BvhNode));
  if (!orec.empty()) std::memcpy(&host[o_or], orec.data(), orec.size() * sizeof(OtherRec));
  if (!lbvh.empty()) std::memcpy(&host[o_lb], lbvh.data(), lbvh.size() * sizeof(BvhNode));
  if (!lclus.empty()) std::memcpy(&host[o_cc], lclus.data(), lclus.size() * sizeof(ConeCluster));
  if (!lcone.empty()) std::memcpy(&host[o_lm], lcone.data(), lcone.size() * sizeof(int32_t));
  if (!line_rec.empty()) std::memcpy(&host[o_lr], line_rec.data(), line_rec.size() * sizeof(QuadRec));
  if (!fx_gen.empty()) std::memcpy(&host[o_fg], fx_gen.data(), fx_gen.size() * sizeof(SphereGen));
  if (!fx_quads.empty()) std::memcpy(&host[o_fq], fx_quads.data(), fx_quads.size() * sizeof(QuadRec));
  if (!shade.empty()) std::memcpy(&host[o_sh], shade.data(), shade.size() * sizeof(ShadeRec));
  for (size_t i = 0; i < shade.size(); ++i) {
    const double rt2[2] = {shade[i].reflective, shade[i].transparency};
    std::memcpy(&host[o_rt + i * 2 * sizeof(double)], rt2, sizeof rt2);
  }
  if (!lrec.empty()) std::memcpy(&host[o_li], lrec.data(), lrec.size() * sizeof(LightRec));
  if (!grec.empty()) std::memcpy(&host[o_gr], grec.data(), grec.size() * sizeof(GroupRec));
  if (!lb.cells.empty()) {
    std::memcpy(&host[o_lc], lb.cells.data(), lb.cells.size() * sizeof(LbCell));
    if (!lb.ov.empty()) std::memcpy(&host[o_lv], lb.ov.data(), lb.ov.size() * sizeof(uint16_t));
    std::memcpy(&host[o_ld], lb.delta.data(), lb.delta.size() * sizeof(float));
    std::memcpy(&host[o_ll], lb.limit.data(), lb.limit.size() * sizeof(float));
  }

  rt_scene* s = new rt_scene();
  s->device = device;
  // children per ray at most (WfSizing::branch): the exact bound of the arenas
  int branch = 0;
  for (size_t i = 0; i < n_shapes; ++i)
    branch = std::max(branch, (shapes[i].reflective != 0.0 ? 1 : 0) + (shapes[i].transparency != 0.0 ? 1 : 0));
  s->sizing.branch = branch;
  s->band_sizing.branch = branch;
  {
    std::lock_guard<std::mutex> tlk(g_tune_mu);
    s->tune = g_tune_defaults;
  }
  auto cleanup = [&](int rc) {
    rt_scene_destroy(s);
    return rc;
  };
  int rc;
  DeviceGuard restore;  // the caller's device, whatever happens below
  if ((rc = [&]() -> int {
         RT_HIP(hipSetDevice(device));
         RT_HIP(hipMalloc(&s->d_blob, total));
         RT_HIP(hipMemcpy(s->d_blob, host.data(), total, hipMemcpyHostToDevice));
         RT_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
         return RT_OK;
       }()) != RT_OK)
    return cleanup(rc);
  unsigned char* b = (unsigned char*)s->d_blob;
  s->dev.sph_diag = (const SphereDiag*)(b + o_diag);
  s->dev.sph_gen = (const SphereGen*)(b + o_gen);
  s->dev.planes = (const PlaneRec*)(b + o_pl);
  s->dev.quads = (const QuadRec*)(b + o_qd);
  s->dev.bvh = bvh.empty() ? nullptr : (const BvhNode*)(b + o_bv);
  s->dev.bvh_pair = bvh_pair.empty() ? nullptr : (const BvhPair*)(b + o_bp);
  s->dev.bvhw = bvh_wide.empty() ? nullptr : (const BvhWide*)(b + o_bw);
  s->dev.bvhw16 = bvh_wide16.empty() ? nullptr : (const BvhWide16*)(b + o_bh);
  s->dev.n_bvhw = (int32_t)bvh_wide.size();
  s->dev.bvhw_stack = wide_stack;
  s->dev.n_bvh = (int32_t)bvh.size();
  s->dev.bvh_depth = bvh_depth;
  s->dev.obvh = obvh.empty() ? nullptr : (const BvhNode*)(b + o_ob);
  s->dev.orec = (const OtherRec*)(b + o_or);
  s->dev.lbvh = lbvh.empty() ? nullptr : (const BvhNode*)(b + o_lb);
  s->dev.lclus = (const ConeCluster*)(b + o_cc);
  s->dev.lcone = (const int32_t*)(b + o_lm);
  s->dev.n_lclus = (int32_t)lclus.size();
  s->dev.lrec = (const QuadRec*)(b + o_lr);
  s->dev.n_lbvh = (int32_t)lbvh.size();
  s->dev.n_lrec = (int32_t)line_rec.size();
  s->dev.n_obvh = (int32_t)obvh.size();
  s->dev.obvh_depth = obvh_depth;
  s->dev.n_orec = (int32_t)orec.size();
  s->dev.fx_gen = (const SphereGen*)(b + o_fg);
  s->dev.fx_quads = (const QuadRec*)(b + o_fq);
  s->dev.n_fx_gen = (int32_t)fx_gen.size();
  s->dev.n_fx_quads = (int32_t)fx_quads.size();
  s->dev.lb_cells = lb.cells.empty() ? nullptr : (const LbCell*)(b + o_lc);
  s->dev.lb_ov = (const uint16_t*)(b + o_lv);
  s->dev.lb_delta = (const float*)(b + o_ld);
  s->dev.lb_limit = (const float*)(b + o_ll);
  s->dev.lb_res = lb.res;
  s->dev.lb_n_items = (int32_t)std::min<size_t>(lb.n_items, 0x7FFFFFFF);
  s->dev.shade = (const ShadeRec*)(b + o_sh);
  s->dev.refl_transp = (const double*)(b + o_rt);
  s->dev.lights = (const LightRec*)(b + o_li);
  s->dev.groups = (const GroupRec*)(b + o_gr);
  s->dev.n_groups = (int32_t)n_groups;
  s->dev.n_diag = (int32_t)diag.size();
  s->dev.n_gen = (int32_t)gen.size();
  s->dev.n_planes = (int32_t)planes.size();
  s->dev.n_quads = (int32_t)quads.size();
  s->dev.n_objects = (int32_t)n_shapes;
  s->dev.n_lights = (int32_t)n_lights;
  s->n_objects = (int)n_shapes;
  s->n_lights = (int)n_lights;
  *out = s;
  return RT_OK;
  });
}

void rt_scene_destroy(rt_scene* s) {
  if (!s) return;
  DeviceGuard restore(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  s->multi.release();
  (void)hipSetDevice(s->device);
  if (s->d_blob) (void)hipFree(s->d_blob);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;  // the host contexts and workspaces release their memory (on the scene's device)
}

uint32_t rt_shard_rows(uint32_t vsize, uint32_t row_block, uint32_t shard, uint32_t n_shards) {
  if (row_block == 0 || n_shards == 0 || shard >= n_shards) return 0;
  uint32_t rows = 0;
  for (uint32_t blk = shard; (uint64_t)blk * row_block < vsize; blk += n_shards) {
    uint32_t y0 = blk * row_block;
    rows += std::min(row_block, vsize - y0);
  }
  return rows;
}

int rt_render_shard_device(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth,
                           uint32_t aa_samples, uint32_t row_block, uint32_t shard, uint32_t n_shards,
                           double* d_out_rgb, void* stream, rt_stats* stats) {
  return guarded([&]() -> int {
  return rt_render_shard_device_ex(scene, camera, max_depth, aa_samples, row_block, shard, n_shards, 0, d_out_rgb,
                                   stream, stats);
  });
}

int rt_render_shard_device_ex(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth,
                              uint32_t aa_samples, uint32_t row_block, uint32_t shard, uint32_t n_shards,
                              uint32_t flags, double* d_out_rgb, void* stream, rt_stats* stats) {
  return guarded([&]() -> int {
  if (!scene || !camera || !d_out_rgb) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (row_block == 0 || n_shards == 0 || shard >= n_shards)
    return fail(RT_ERR_INVALID_ARGUMENT, "bad shard specification");
  if (camera->hsize == 0 || camera->vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty camera");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::unique_lock<std::mutex> lk(s->mu);
  auto t0 = std::chrono::steady_clock::now();
  RT_DEVICE(s->device);
  const uint32_t rows = rt_shard_rows(camera->vsize, row_block, shard, n_shards);
  const uint64_t n_tasks = (uint64_t)rows * camera->hsize * aa_samples;
  if (n_tasks >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "shard too large");
  hipStream_t st = (hipStream_t)stream;  // NULL = the default stream (torch's current stream is often 0)
  DevStats ds{};
  float ms = 0.f;
  int rc = run_render(s, to_dev_camera(*camera), nullptr, (uint32_t)n_tasks, aa_samples, max_depth, row_block, shard,
                      n_shards, d_out_rgb, st, stats ? &ds : nullptr, stats ? &ms : nullptr, flags, nullptr, nullptr,
                      1, false, &lk);
  if (rc != RT_OK) return rc;
  if (stats)
    fill_stats(stats, ds, ms, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return RT_OK;
  });
}

static bool valid_pattern(uint32_t period, uint64_t mask) {
  return period >= 1 && period <= 64 && mask != 0 && (period == 64 || (mask >> period) == 0);
}

uint32_t rt_pattern_rows(uint32_t vsize, uint32_t row_block, uint32_t period, uint64_t mask) {
  if (row_block == 0 || !valid_pattern(period, mask)) return 0;
  uint32_t rows = 0;
  for (uint64_t blk = 0; blk * row_block < vsize; ++blk)
    if ((mask >> (blk % period)) & 1u) rows += std::min<uint32_t>(row_block, vsize - (uint32_t)(blk * row_block));
  return rows;
}

namespace {
// rt_render_frames_device (blk_period 0: shard `shard` of `n_shards`) and
// rt_render_block_pattern_device (the blocks of a period pattern).
int render_frames(const rt_scene* scene, const rt_camera_desc* cameras, uint32_t n_frames, uint32_t max_depth,
                  uint32_t aa_samples, uint32_t row_block, uint32_t shard, uint32_t n_shards, uint32_t blk_period,
                  uint64_t blk_mask, uint32_t flags, double* const* d_out_rgb, void* stream, rt_stats* stats) {
  if (!scene || (n_frames && (!cameras || !d_out_rgb))) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (row_block == 0 || n_shards == 0 || shard >= n_shards)
    return fail(RT_ERR_INVALID_ARGUMENT, "bad shard specification");
  if (blk_period && !valid_pattern(blk_period, blk_mask))
    return fail(RT_ERR_INVALID_ARGUMENT, "bad block pattern (period 1..64, a non-empty mask below 2^period)");
  if (!valid_aa(aa_samples)) return fail(RT_ERR_INVALID_ARGUMENT, "aa_samples must be 1, 2, 4, 8 or 16");
  for (uint32_t f = 0; f < n_frames; ++f) {
    if (!d_out_rgb[f]) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
    if (cameras[f].hsize == 0 || cameras[f].vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty camera");
    if (cameras[f].hsize != cameras[0].hsize || cameras[f].vsize != cameras[0].vsize)
      return fail(RT_ERR_INVALID_ARGUMENT, "the frames of a batch must share hsize and vsize");
  }
  if (n_frames == 0) {
    if (stats) std::memset(stats, 0, sizeof *stats);
    return RT_OK;
  }
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::unique_lock<std::mutex> lk(s->mu);
  auto t0 = std::chrono::steady_clock::now();
  RT_DEVICE(s->device);
  const uint32_t rows = blk_period ? rt_pattern_rows(cameras[0].vsize, row_block, blk_period, blk_mask)
                                  : rt_shard_rows(cameras[0].vsize, row_block, shard, n_shards);
  const uint64_t per = (uint64_t)rows * cameras[0].hsize * aa_samples;
  const uint64_t padded = (per + 63) & ~(uint64_t)63;
  if (padded >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "shard too large");
  hipStream_t st = (hipStream_t)stream;
  // one pass of the generation pipeline per group of kMaxFrames frames; a
  // render that cannot batch (counted, or a scene without the fast path's
  // hierarchies) goes frame by frame, with the counters summed
  const bool batch = !stats && !(flags & RT_RENDER_EXHAUSTIVE) && s->tune.accel != 0 &&
                     (s->dev.n_bvh > 0 || s->dev.n_obvh > 0 || s->dev.n_lbvh > 0) && per > 0;
  DevStats sum{};
  float ms_sum = 0.f;
  // a pass holds at most ~2^25 root rays (16 C3 frames; 2 C5 frames), which bounds the
  // workspace's queues; larger frames gain nothing from sharing launches
  const uint32_t per_pass = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kMaxFrames, ((uint64_t)1 << 25) / std::max<uint64_t>(padded, 1)));
  for (uint32_t f0 = 0; f0 < n_frames;) {
    const uint32_t nf = batch ? std::min<uint32_t>(per_pass, n_frames - f0) : 1u;
    FrameTable tab{};
    for (uint32_t f = 0; f < nf; ++f) {
      tab.cam[f] = to_dev_camera(cameras[f0 + f]);
      tab.out[f] = d_out_rgb[f0 + f];
    }
    DevStats ds{};
    float ms = 0.f;
    int rc = run_render(s, tab.cam[0], nullptr, (uint32_t)per, aa_samples, max_depth, row_block, shard, n_shards,
                        tab.out[0], st, stats ? &ds : nullptr, stats ? &ms : nullptr, flags, nullptr,
                        nf > 1 ? &tab : nullptr, nf, false, &lk, false, false, blk_period, blk_mask);
    if (rc != RT_OK) return rc;
    if (stats) {
      sum.rays_primary += ds.rays_primary; sum.rays_reflect += ds.rays_reflect;
      sum.rays_refract += ds.rays_refract; sum.rays_shadow += ds.rays_shadow;
      sum.rays_shadow_traced += ds.rays_shadow_traced; sum.sphere_tests += ds.sphere_tests;
      sum.plane_tests += ds.plane_tests; sum.other_tests += ds.other_tests;
      sum.sphere_tests_executed += ds.sphere_tests_executed; sum.box_tests_executed += ds.box_tests_executed;
      sum.exhaustive = ds.exhaustive;
      sum.sphere_disc_ge0 = ds.exhaustive ? sum.sphere_disc_ge0 + ds.sphere_disc_ge0 : ds.sphere_disc_ge0;
      ms_sum += ms;
    }
    f0 += nf;
  }
  if (stats)
    fill_stats(stats, sum, ms_sum, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return RT_OK;
}
}  // namespace

int rt_render_frames_device(const rt_scene* scene, const rt_camera_desc* cameras, uint32_t n_frames,
                            uint32_t max_depth, uint32_t aa_samples, uint32_t row_block, uint32_t shard,
                            uint32_t n_shards, double* const* d_out_rgb, void* stream, rt_stats* stats) {
  return guarded([&]() -> int {
  return render_frames(scene, cameras, n_frames, max_depth, aa_samples, row_block, shard, n_shards, 0, 0, 0,
                       d_out_rgb, stream, stats);
  });
}

int rt_render_block_pattern_device(const rt_scene* scene, const rt_camera_desc* cameras, uint32_t n_frames,
                                   uint32_t max_depth, uint32_t aa_samples, uint32_t row_block, uint32_t period,
                                   uint64_t mask, uint32_t flags, double* const* d_out_rgb, void* stream,
                                   rt_stats* stats) {
  return guarded([&]() -> int {
  if (period == 0) return fail(RT_ERR_INVALID_ARGUMENT, "bad block pattern (period 1..64)");
  if (flags & ~(uint32_t)RT_RENDER_EXHAUSTIVE) return fail(RT_ERR_INVALID_ARGUMENT, "unknown render flags");
  return render_frames(scene, cameras, n_frames, max_depth, aa_samples, row_block, 0, 1, period, mask, flags,
                       d_out_rgb, stream, stats);
  });
}

namespace {
// `Camera::render` into a host canvas with the device-to-host copy overlapped
// (rt_render_ex): the frame's rows are cut into `bands`
// contiguous bands of 64-block patterns (rt_render_block_pattern_device's
// mapping with one period over the whole canvas). Band k renders on its own
// stream (its own workspace), starting when band k-1's render is done, so the
// GPU works on one band at a time as in a whole-frame render, and band k's copy
// to the host runs behind its render while band k+1 renders. Every pixel is
// that of the whole-frame render (a pattern only chooses which rows a render
// owns). The caller's canvas must be pinned (rt_host_buffer_alloc) or
// registrable for the call (d2h = 1); RT_ERR_NO_DEVICE asks the caller for
// the one-render path. A band that overflowed its arenas is rendered again,
// synchronously, before the call returns (every synchronous call returns a
// complete frame).
int render_banded(rt_scene* s, std::unique_lock<std::mutex>& lk, rt_scene::HostCtx* c, const rt_camera_desc& cam,
                  uint32_t max_depth, uint32_t aa, double* out_rgb) {
  const uint32_t W = cam.hsize, H = cam.vsize;
  const int bands = std::max(2, std::min(kMaxBands, s->tune.bands));
  const uint32_t rb = (H + 63) / 64, nb = (H + rb - 1) / rb;  // nb <= 64 blocks of rb rows: one period
  if (nb < (uint32_t)bands * 2) return RT_ERR_NO_DEVICE;
  // band k = blocks [b[k], b[k+1]): the first band takes band_pct of the rows, the
  // others share the remainder in sizes falling by band_ratio percent per band
  uint32_t b[kMaxBands + 1] = {};
  b[1] = std::max<uint32_t>(1, std::min<uint32_t>(nb - (uint32_t)bands + 1, (uint32_t)((uint64_t)nb * s->tune.band_pct / 100)));
  {
    double wsum = 0.0, wk = 1.0;
    for (int k = 1; k < bands; ++k, wk *= s->tune.band_ratio / 100.0) wsum += wk;
    double acc = 0.0;
    wk = 1.0;
    for (int k = 2; k < bands; ++k, wk *= s->tune.band_ratio / 100.0) {
      acc += wk;
      const uint32_t at = b[1] + (uint32_t)((nb - b[1]) * acc / wsum + 0.5);
      b[k] = std::min<uint32_t>(nb - (uint32_t)(bands - k), std::max<uint32_t>(b[k - 1] + 1, at));
    }
  }
  b[bands] = nb;
  const size_t bytes = (size_t)W * H * 3 * sizeof(double);
  bool registered = false;
  if (!pinned_block(out_rgb, bytes)) {
    if (s->tune.d2h != 1 || hipHostRegister(out_rgb, bytes, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return RT_ERR_NO_DEVICE;  // (a buffer the DMA engine cannot write: the one-render path stages it)
    }
    registered = true;
  }
  struct Unregister {
    void* p;
    bool on;
    ~Unregister() {
      if (on && hipHostUnregister(p) != hipSuccess) (void)hipGetLastError();
    }
  } unreg{out_rgb, registered};
  hipStream_t st[kMaxBands] = {c->stream};
  for (int k = 1; k < bands; ++k) {
    if (!c->band_stream[k - 1]) RT_HIP(hipStreamCreateWithFlags(&c->band_stream[k - 1], hipStreamNonBlocking));
    st[k] = c->band_stream[k - 1];
  }
  for (int k = 0; k < bands; ++k)
    if (!c->band_ev[k]) RT_HIP(hipEventCreateWithFlags(&c->band_ev[k], hipEventDisableTiming));
  const DevCamera dc = to_dev_camera(cam);
  const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
  rt_scene::WfSlot* used[kMaxBands] = {};
  auto unpin = [&](int k) {
    if (used[k]) {
      --used[k]->pins;
      used[k] = nullptr;
    }
  };
  struct UnpinAll {
    std::function<void()> f;
    ~UnpinAll() { f(); }
  } unpin_all{[&]() {
    if (!lk.owns_lock()) lk.lock();
    for (int k = 0; k < bands; ++k) unpin(k);
  }};
  uint32_t y0[kMaxBands + 1];
  for (int k = 0; k <= bands; ++k) y0[k] = std::min(H, b[k] * rb);
  auto mask_of = [&](int k) {
    const uint64_t below_end = b[k + 1] >= 64 ? ~0ull : ((1ull << b[k + 1]) - 1ull);
    const uint64_t below_start = (1ull << b[k]) - 1ull;
    return all & below_end & ~below_start;
  };
  for (int k = 0; k < bands; ++k) {
    if (k > 0) RT_HIP(hipStreamWaitEvent(st[k], c->band_ev[k - 1], 0));  // band k after band k-1's render
    const uint32_t rows = y0[k + 1] - y0[k];
    // band k+1 starts after band k's render, or (band_gen >= 0) after its generation band_gen's launch
    const bool early = s->tune.band_gen >= 0 && k + 1 < bands;
    bool recorded = false;
    int rc = run_render(s, dc, nullptr, rows * W * aa, aa, max_depth, rb, 0, 1, c->d_out + (size_t)y0[k] * W * 3, st[k],
                        nullptr, nullptr, 0, &used[k], nullptr, 1, false, &lk, false, true, nb, mask_of(k),
                        early ? c->band_ev[k] : nullptr, s->tune.band_gen, &recorded, &s->band_sizing);
    if (rc != RT_OK) return rc;
    if (!recorded) RT_HIP(hipEventRecord(c->band_ev[k], st[k]));
    RT_HIP(hipMemcpyAsync(out_rgb + (size_t)y0[k] * W * 3, c->d_out + (size_t)y0[k] * W * 3,
                          (size_t)rows * W * 3 * sizeof(double), hipMemcpyDeviceToHost, st[k]));
  }
  lk.unlock();  // the workspaces stay pinned to this call
  for (int k = 0; k < bands; ++k) RT_HIP(hipStreamSynchronize(st[k]));
  lk.lock();
  for (int k = 0; k < bands; ++k) {
    if (!used[k]) continue;
    used[k]->wf->learn(s->band_sizing);
    bool over = false;
    RT_HIP(used[k]->wf->take_overflow(&over));
    unpin(k);
    if (!over) continue;
    // (its canvas rows are NaN: render the band again, synchronously, with the arenas grown)
    const uint32_t rows = y0[k + 1] - y0[k];
    int rc = run_render(s, dc, nullptr, rows * W * aa, aa, max_depth, rb, 0, 1, c->d_out + (size_t)y0[k] * W * 3,
                        st[k], nullptr, nullptr, 0, nullptr, nullptr, 1, true, &lk, false, false, nb, mask_of(k),
                        nullptr, -1, nullptr, &s->band_sizing);
    if (rc != RT_OK) return rc;
    RT_HIP(hipMemcpyAsync(out_rgb + (size_t)y0[k] * W * 3, c->d_out + (size_t)y0[k] * W * 3,
                          (size_t)rows * W * 3 * sizeof(double), hipMemcpyDeviceToHost, st[k]));
    lk.unlock();
    const hipError_t e = hipStreamSynchronize(st[k]);
    lk.lock();
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("banded render: ") + hipGetErrorString(e));
  }
  return RT_OK;
}
}  // namespace

int rt_render_aa(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth, uint32_t aa_samples,
                 double* out_rgb, rt_stats* stats) {
  return guarded([&]() -> int {
  return rt_render_ex(scene, camera, max_depth, aa_samples, 0, out_rgb, stats);
  });
}

int rt_render_ex(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth, uint32_t aa_samples,
                 uint32_t flags, double* out_rgb, rt_stats* stats) {
  return guarded([&]() -> int {
  if (!scene || !camera || !out_rgb) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (camera->hsize == 0 || camera->vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty camera");
  if (!valid_aa(aa_samples)) return fail(RT_ERR_INVALID_ARGUMENT, "aa_samples must be 1, 2, 4, 8 or 16");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::unique_lock<std::mutex> lk(s->mu);
  auto t0 = std::chrono::steady_clock::now();
  RT_DEVICE(s->device);
  const uint64_t n_pix = (uint64_t)camera->hsize * camera->vsize;
  if (n_pix * aa_samples >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "canvas too large for one launch");
  CtxLease cx{s, lk};
  RT_TAKE_CTX(cx);
  int rc = ensure_dev_buffer(&cx.c->d_out, &cx.c->out_cap, n_pix * 3);
  if (rc != RT_OK) return rc;
  // a large frame without counters: bands, each band's copy behind its render (render_banded)
  if (!stats && flags == 0 && s->tune.bands > 1 && s->tune.accel != 0 && (s->dev.n_bvh > 0 || s->dev.n_obvh > 0 || s->dev.n_lbvh > 0) &&
      n_pix * aa_samples >= ((uint64_t)1 << 20)) {
    rc = render_banded(s, lk, cx.c, *camera, max_depth, aa_samples, out_rgb);
    if (rc != RT_ERR_NO_DEVICE) return rc;  // (RT_ERR_NO_DEVICE: not bandable, render it whole below)
  }
  DevStats ds{};
  float ms = 0.f;
  rc = run_render(s, to_dev_camera(*camera), nullptr, (uint32_t)(n_pix * aa_samples), aa_samples, max_depth,
                  camera->vsize, 0, 1, cx.c->d_out, cx.c->stream, stats ? &ds : nullptr, &ms, flags, nullptr, nullptr,
                  1, true, &lk);
  if (rc != RT_OK) return rc;
  const int d2h = s->tune.d2h;
  lk.unlock();  // the copy to the caller's canvas runs unlocked (the context is this call's)
  if ((rc = copy_to_host(cx.c, d2h, out_rgb, cx.c->d_out, n_pix * 3 * sizeof(double), cx.c->stream)) != RT_OK)
    return rc;
  if (stats)
    fill_stats(stats, ds, ms, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return RT_OK;
  });
}

int rt_render_ppm(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth, uint32_t aa_samples,
                  char* out, size_t cap, size_t* out_len, rt_stats* stats) {
  return guarded([&]() -> int {
  if (!scene || !camera || !out_len) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (camera->hsize == 0 || camera->vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty camera");
  if (!valid_aa(aa_samples)) return fail(RT_ERR_INVALID_ARGUMENT, "aa_samples must be 1, 2, 4, 8 or 16");
  if (camera->hsize > kPpmMaxWidth)
    return fail(RT_ERR_INVALID_ARGUMENT, "canvas wider than the device PPM encoder's row (use rt_canvas_to_ppm)");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::unique_lock<std::mutex> lk(s->mu);
  auto t0 = std::chrono::steady_clock::now();
  RT_DEVICE(s->device);
  const uint32_t W = camera->hsize, H = camera->vsize;
  const uint64_t n_pix = (uint64_t)W * H;
  if (n_pix * aa_samples >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "canvas too large for one launch");
  CtxLease cx{s, lk};
  RT_TAKE_CTX(cx);
  rt_scene::HostCtx* c = cx.c;
  int rc = ensure_dev_buffer(&c->d_out, &c->out_cap, n_pix * 3);
  if (rc != RT_OK) return rc;
  const PpmHeader hd = ppm_header(W, H);
  const size_t bound = hd.n + (size_t)12 * n_pix + H;  // <= 4 bytes per component, one '\n' per row
  if (c->ppm_cap < bound) {
    if (c->d_ppm) (void)hipFree(c->d_ppm);
    c->d_ppm = nullptr;
    c->ppm_cap = 0;
    RT_HIP(hipMalloc(&c->d_ppm, bound));
    c->ppm_cap = bound;
  }
  if (c->ppm_rows_cap < H) {
    if (c->d_ppm_rows) (void)hipFree(c->d_ppm_rows);
    c->d_ppm_rows = nullptr;
    c->ppm_rows_cap = 0;
    RT_HIP(hipMalloc(&c->d_ppm_rows, (size_t)H * 4 + ((size_t)H + 1) * 8 + 8));
    c->ppm_rows_cap = H;
  }
  unsigned long long* d_off = (unsigned long long*)(((uintptr_t)c->d_ppm_rows + (size_t)H * 4 + 7) & ~(uintptr_t)7);
  DevStats ds{};
  float ms = 0.f;
  rc = run_render(s, to_dev_camera(*camera), nullptr, (uint32_t)(n_pix * aa_samples), aa_samples, max_depth, H, 0,
                  1, c->d_out, c->stream, stats ? &ds : nullptr, stats ? &ms : nullptr, 0, nullptr, nullptr, 1, true,
                  &lk);
  if (rc != RT_OK) return rc;
  const int d2h = s->tune.d2h;
  lk.unlock();
  RT_HIP(ppm_encode_device(c->d_out, W, H, c->d_ppm, c->ppm_cap, (unsigned*)c->d_ppm_rows, d_off, hd, c->stream));
  unsigned long long body = 0;
  RT_HIP(hipMemcpyAsync(&body, d_off + H, sizeof body, hipMemcpyDeviceToHost, c->stream));
  RT_HIP(hipStreamSynchronize(c->stream));
  *out_len = hd.n + (size_t)body;
  if (out) {
    if (cap < *out_len) return fail(RT_ERR_BUFFER_TOO_SMALL, "PPM buffer too small");
    if ((rc = copy_to_host(c, d2h, out, c->d_ppm, *out_len, c->stream)) != RT_OK) return rc;
  }
  if (stats)
    fill_stats(stats, ds, ms, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return RT_OK;
  });
}

int rt_canvas_to_ppm_device(const double* d_rgb, uint32_t width, uint32_t height, char* d_out, size_t cap,
                            size_t* out_len, void* stream) {
  return guarded([&]() -> int {
  if (!out_len || (width && height && !d_rgb)) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (width > kPpmMaxWidth)
    return fail(RT_ERR_INVALID_ARGUMENT, "canvas wider than the device PPM encoder's row (use rt_canvas_to_ppm)");
  const PpmHeader hd = ppm_header(width, height);
  if (height == 0) {  // the header alone (ppm.rs:24-27)
    *out_len = hd.n;
    if (d_out && cap >= hd.n) RT_HIP(hipMemcpyAsync(d_out, hd.s, hd.n, hipMemcpyHostToDevice, (hipStream_t)stream));
    RT_HIP(hipStreamSynchronize((hipStream_t)stream));
    return d_out && cap < hd.n ? fail(RT_ERR_BUFFER_TOO_SMALL, "PPM buffer too small") : RT_OK;
  }
  hipStream_t st = (hipStream_t)stream;
  void* rows = nullptr;
  RT_HIP(hipMallocAsync(&rows, (size_t)height * 4 + ((size_t)height + 1) * 8 + 8, st));
  unsigned long long* d_off = (unsigned long long*)(((uintptr_t)rows + (size_t)height * 4 + 7) & ~(uintptr_t)7);
  hipError_t e = ppm_encode_device(d_rgb, width, height, d_out, cap, (unsigned*)rows, d_off, hd, st);
  unsigned long long body = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&body, d_off + height, sizeof body, hipMemcpyDeviceToHost, st);
  (void)hipFreeAsync(rows, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("rt_canvas_to_ppm_device: ") + hipGetErrorString(e));
  *out_len = hd.n + (size_t)body;
  if (d_out && cap < *out_len) return fail(RT_ERR_BUFFER_TOO_SMALL, "PPM buffer too small");
  return RT_OK;
  });
}

int rt_render(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth, double* out_rgb,
              rt_stats* stats) {
  return guarded([&]() -> int {
  return rt_render_aa(scene, camera, max_depth, 1, out_rgb, stats);
  });
}

int rt_color_at_batch(const rt_scene* scene, const double* rays, size_t n, uint32_t remaining,
                      double* out_rgb, rt_stats* stats) {
  return guarded([&]() -> int {
  return rt_color_at_batch_ex(scene, rays, n, remaining, 0, out_rgb, stats);
  });
}

int rt_color_at_batch_ex(const rt_scene* scene, const double* rays, size_t n, uint32_t remaining, uint32_t flags,
                         double* out_rgb, rt_stats* stats) {
  return guarded([&]() -> int {
  if (!scene || (n && (!rays || !out_rgb))) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (n >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "batch too large");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::unique_lock<std::mutex> lk(s->mu);
  auto t0 = std::chrono::steady_clock::now();
  RT_DEVICE(s->device);
  CtxLease cx{s, lk};
  RT_TAKE_CTX(cx);
  rt_scene::HostCtx* c = cx.c;
  int rc = ensure_dev_buffer(&c->d_in, &c->in_cap, n * 6);
  if (rc != RT_OK) return rc;
  rc = ensure_dev_buffer(&c->d_out, &c->out_cap, n * 3);
  if (rc != RT_OK) return rc;
  if (n) RT_HIP(hipMemcpyAsync(c->d_in, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  DevCamera cam{};
  DevStats ds{};
  float ms = 0.f;
  rc = run_render(s, cam, c->d_in, (uint32_t)n, 1, remaining, 1, 0, 1, c->d_out, c->stream, stats ? &ds : nullptr,
                  &ms, flags, nullptr, nullptr, 1, true, &lk);
  if (rc != RT_OK) return rc;
  lk.unlock();
  if (n) RT_HIP(hipMemcpyAsync(out_rgb, c->d_out, n * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  RT_HIP(hipStreamSynchronize(c->stream));
  if (stats)
    fill_stats(stats, ds, ms, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return RT_OK;
  });
}

int rt_is_shadowed_batch(const rt_scene* scene, const double* points, size_t n, uint32_t light,
                         uint8_t* out) {
  return guarded([&]() -> int {
  if (!scene || (n && (!points || !out))) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  rt_scene* s = const_cast<rt_scene*>(scene);
  if ((int)light >= s->n_lights) return fail(RT_ERR_INVALID_ARGUMENT, "light index out of range");
  if (n >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "batch too large");
  std::unique_lock<std::mutex> lk(s->mu);
  RT_DEVICE(s->device);
  if (n == 0) return RT_OK;
  CtxLease cx{s, lk};
  RT_TAKE_CTX(cx);
  rt_scene::HostCtx* c = cx.c;
  lk.unlock();  // the context is this call's: nothing below touches shared state
  int rc = ensure_dev_buffer(&c->d_in, &c->in_cap, n * 3);
  if (rc != RT_OK) return rc;
  rc = ensure_dev_buffer(&c->d_out, &c->out_cap, (n + 7) / 8);
  if (rc != RT_OK) return rc;
  RT_HIP(hipMemcpyAsync(c->d_in, points, n * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  RT_HIP(launch_shadow(s->dev, c->d_in, (int)n, (int)light, (uint8_t*)c->d_out, c->stream));
  RT_HIP(hipMemcpyAsync(out, c->d_out, n, hipMemcpyDeviceToHost, c->stream));
  RT_HIP(hipStreamSynchronize(c->stream));
  return RT_OK;
  });
}

int rt_hit_batch(const rt_scene* scene, const double* rays, size_t n, double* out24) {
  return guarded([&]() -> int {
  if (!scene || (n && (!rays || !out24))) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (n >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "batch too large");
  rt_scene* s = const_cast<rt_scene*>(scene);
  std::unique_lock<std::mutex> lk(s->mu);
  RT_DEVICE(s->device);
  if (n == 0) return RT_OK;
  CtxLease cx{s, lk};
  RT_TAKE_CTX(cx);
  rt_scene::HostCtx* c = cx.c;
  lk.unlock();
  int rc = ensure_dev_buffer(&c->d_in, &c->in_cap, n * 6);
  if (rc != RT_OK) return rc;
  rc = ensure_dev_buffer(&c->d_out, &c->out_cap, n * 24);
  if (rc != RT_OK) return rc;
  RT_HIP(hipMemcpyAsync(c->d_in, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  RT_HIP(launch_hit(s->dev, c->d_in, (int)n, c->d_out, c->stream));
  RT_HIP(hipMemcpyAsync(out24, c->d_out, n * 24 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  RT_HIP(hipStreamSynchronize(c->stream));
  return RT_OK;
  });
}

// Single-process multi-GPU render (the GPU form of `render_multithreaded`,
// camera.rs:150-217): interleaved row blocks, one RCCL gather to device 0.
// The communicators and device buffers are cached on scenes[0] across calls
// (rt_scene::MultiCache) and rebuilt only when the scene set changes.
int rt_render_multi(rt_scene* const* scenes, int n_devices, const rt_camera_desc* camera,
                    uint32_t max_depth, uint32_t aa_samples, uint32_t row_block, double* out_rgb,
                    rt_stats* stats) {
  return guarded([&]() -> int {
  if (!scenes || n_devices < 1 || !camera || !out_rgb || row_block == 0)
    return fail(RT_ERR_INVALID_ARGUMENT, "bad arguments");
  if (camera->hsize == 0 || camera->vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty camera");
  if (!valid_aa(aa_samples)) return fail(RT_ERR_INVALID_ARGUMENT, "aa_samples must be 1, 2, 4, 8 or 16");
  for (int i = 0; i < n_devices; ++i)
    if (!scenes[i] || scenes[i]->device != i)
      return fail(RT_ERR_INVALID_ARGUMENT, "scenes[i] must live on device i");
  auto t0 = std::chrono::steady_clock::now();
  DeviceGuard restore;  // the caller's device (the loops below visit every device)
  const uint32_t W = camera->hsize, H = camera->vsize;
  uint32_t max_rows = 0;
  for (int i = 0; i < n_devices; ++i) max_rows = std::max(max_rows, rt_shard_rows(H, row_block, i, n_devices));
  if ((uint64_t)max_rows * W * aa_samples >= (1ull << 31))
    return fail(RT_ERR_INVALID_ARGUMENT, "shard too large for one launch");
  const size_t per = (size_t)max_rows * W * 3;  // padded per-rank element count
  rt_scene* s0 = scenes[0];
  std::lock_guard<std::mutex> mlk(s0->multi_mu);
  rt_scene::MultiCache& mc = s0->multi;
  const std::vector<rt_scene*> want(scenes, scenes + n_devices);
  if (mc.scenes != want) {
    mc.release();
    mc.scenes = want;
    mc.send.assign(n_devices, nullptr);
    mc.send_cap.assign(n_devices, 0);
    if (n_devices > 1) {
      std::vector<int> devs(n_devices);
      for (int i = 0; i < n_devices; ++i) devs[i] = i;
      mc.comms.assign(n_devices, nullptr);
      if (ncclCommInitAll(mc.comms.data(), n_devices, devs.data()) != ncclSuccess) {
        mc.comms.clear();
        mc.scenes.clear();
        return fail(RT_ERR_RCCL, "ncclCommInitAll failed");
      }
    }
  }
  mc.ev0.resize(n_devices, nullptr);
  mc.ev1.resize(n_devices, nullptr);
  for (int i = 0; i < n_devices; ++i) {
    RT_HIP(hipSetDevice(i));
    int rc = ensure_dev_buffer(&mc.send[i], &mc.send_cap[i], per);
    if (rc != RT_OK) return rc;
    if (!mc.ev0[i]) RT_HIP(hipEventCreate(&mc.ev0[i]));
    if (!mc.ev1[i]) RT_HIP(hipEventCreate(&mc.ev1[i]));
  }
  RT_HIP(hipSetDevice(0));
  int rc = ensure_dev_buffer(&mc.recv, &mc.recv_cap, per * n_devices);
  if (rc != RT_OK) return rc;
  // every device renders its shard (asynchronously, each on its scene's stream); the
  // workspaces this call renders on stay pinned until it has read their overflow
  // records (no other call takes them over, and no other call's records are read)
  std::vector<rt_scene::WfSlot*> used(n_devices, nullptr);
  auto unpin_all = [&]() {
    for (int i = 0; i < n_devices; ++i)
      if (used[i]) {
        std::lock_guard<std::mutex> lk(scenes[i]->mu);
        --used[i]->pins;
        used[i] = nullptr;
      }
  };
  struct Unpin {
    decltype(unpin_all)& f;
    ~Unpin() { f(); }
  } unpin_on_return{unpin_all};
  int attempt = 0;
render_all:
  for (int i = 0; i < n_devices; ++i) {
    RT_HIP(hipSetDevice(i));
    std::lock_guard<std::mutex> lk(scenes[i]->mu);
    const uint32_t rows = rt_shard_rows(H, row_block, i, n_devices);
    if (stats) RT_HIP(hipEventRecord(mc.ev0[i], scenes[i]->stream));
    rc = run_render(scenes[i], to_dev_camera(*camera), nullptr, rows * W * aa_samples, aa_samples, max_depth,
                    row_block, i, n_devices, mc.send[i], scenes[i]->stream, nullptr, nullptr, 0, &used[i], nullptr,
                    1, false, nullptr, stats != nullptr, true);
    if (rc != RT_OK) return rc;
    if (stats) RT_HIP(hipEventRecord(mc.ev1[i], scenes[i]->stream));
  }
  if (n_devices > 1) {
    if (ncclGroupStart() != ncclSuccess) return fail(RT_ERR_RCCL, "ncclGroupStart");
    for (int i = 0; i < n_devices; ++i)
      if (ncclGather(mc.send[i], i == 0 ? mc.recv : nullptr, per, ncclDouble, 0, mc.comms[i], scenes[i]->stream) !=
          ncclSuccess) {
        (void)ncclGroupEnd();
        return fail(RT_ERR_RCCL, "ncclGather");
      }
    if (ncclGroupEnd() != ncclSuccess) return fail(RT_ERR_RCCL, "ncclGroupEnd");
  } else {
    RT_HIP(hipMemcpyAsync(mc.recv, mc.send[0], per * sizeof(double), hipMemcpyDeviceToDevice, scenes[0]->stream));
  }
  // device 0 holds every shard, rank-major: copy each row block straight into its canvas rows
  RT_HIP(hipSetDevice(0));
  for (int i = 0; i < n_devices; ++i) {
    uint32_t lr = 0;
    for (uint32_t blk = (uint32_t)i; (uint64_t)blk * row_block < H; blk += (uint32_t)n_devices) {
      const uint32_t y0 = blk * row_block, nr = std::min(row_block, H - y0);
      RT_HIP(hipMemcpyAsync(out_rgb + (size_t)y0 * W * 3, mc.recv + (size_t)i * per + (size_t)lr * W * 3,
                            (size_t)nr * W * 3 * sizeof(double), hipMemcpyDeviceToHost, scenes[0]->stream));
      lr += nr;
    }
  }
  for (int i = 0; i < n_devices; ++i) {
    RT_HIP(hipSetDevice(i));
    RT_HIP(hipStreamSynchronize(scenes[i]->stream));
  }
  // a shard that overflowed its queue arenas (this call's workspaces only): the arenas
  // have grown, render the frame again
  bool again = false;
  for (int i = 0; i < n_devices; ++i) {
    if (!used[i]) continue;  // an empty shard
    RT_HIP(hipSetDevice(i));
    std::lock_guard<std::mutex> lk(scenes[i]->mu);
    bool was = false;
    used[i]->wf->learn(scenes[i]->sizing);
    RT_HIP(used[i]->wf->take_overflow(&was));
    again = again || was;
  }
  if (again) {
    if (++attempt > 24) return fail(RT_ERR_HIP, "wavefront queue arenas: the frame does not fit");
    unpin_all();  // (the counters are read from the last attempt's workspaces)
    goto render_all;
  }
  if (stats) {
    std::memset(stats, 0, sizeof *stats);
    for (int i = 0; i < n_devices; ++i) {
      if (!used[i]) continue;  // an empty shard
      RT_HIP(hipSetDevice(i));
      std::lock_guard<std::mutex> lk(scenes[i]->mu);
      DevStats ds{};
      RT_HIP(used[i]->wf->read_stats(&ds));
      rt_stats x;
      fill_stats(&x, ds, 0.f, 0.0);
      stats->rays_primary += x.rays_primary; stats->rays_reflect += x.rays_reflect;
      stats->rays_refract += x.rays_refract; stats->rays_shadow += x.rays_shadow;
      stats->sphere_tests += x.sphere_tests; stats->plane_tests += x.plane_tests;
      stats->other_tests += x.other_tests;
      stats->sphere_disc_ge0 = x.sphere_disc_ge0;  // RT_STATS_NOT_COUNTED: the fast path
      stats->rays_shadow_traced += x.rays_shadow_traced;
      stats->sphere_tests_executed += x.sphere_tests_executed;
      stats->box_tests_executed += x.box_tests_executed;
      float ms = 0.f;  // ms_kernel: the slowest device's shard render (HIP events around it)
      RT_HIP(hipEventElapsedTime(&ms, mc.ev0[i], mc.ev1[i]));
      stats->ms_kernel = std::max(stats->ms_kernel, (double)ms);
    }
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return RT_OK;
  });
}

}  // extern "C"
