// rt_workspace.cpp — one render through the scene's workspace pool
// (run_render: a wavefront workspace per stream, overflow detection and
// re-render), the overflow check of earlier asynchronous frames, the
// device-to-host copy into caller memory, and the counters' conversion.
#include "rt_api_internal.hpp"

namespace rtapi {

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
               hipStream_t stream, DevStats* stats_out, float* ms_out, uint32_t flags, rt_scene::WfSlot** used,
               const FrameTable* batch, unsigned n_frames, bool sync, std::unique_lock<std::mutex>* lk, bool count,
               bool keep_pin, uint32_t blk_period, uint64_t blk_mask, hipEvent_t gen_ev, int gen_ev_g,
               bool* gen_ev_recorded, WfSizing* sizing) {
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

void add_stats(DevStats& sum, const DevStats& ds) {
  sum.rays_primary += ds.rays_primary; sum.rays_reflect += ds.rays_reflect;
  sum.rays_refract += ds.rays_refract; sum.rays_shadow += ds.rays_shadow;
  sum.rays_shadow_traced += ds.rays_shadow_traced; sum.sphere_tests += ds.sphere_tests;
  sum.plane_tests += ds.plane_tests; sum.other_tests += ds.other_tests;
  sum.sphere_tests_executed += ds.sphere_tests_executed; sum.box_tests_executed += ds.box_tests_executed;
  sum.exhaustive = ds.exhaustive;
  // (the fast path reports RT_STATS_NOT_COUNTED for disc >= 0: not a sum)
  sum.sphere_disc_ge0 = ds.exhaustive ? sum.sphere_disc_ge0 + ds.sphere_disc_ge0 : ds.sphere_disc_ge0;
}

}  // namespace rtapi
