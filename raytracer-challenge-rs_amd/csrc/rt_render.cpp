// rt_render.cpp — the render entry points of include/rt_render.h:
// `Camera::render` (camera.rs:133-148) into device shards, frame batches and
// block patterns, into a host canvas (row bands with overlapped copies), into
// PPM text (image/ppm.rs:24-51), and the ray-batch entry points
// (`World::color_at`, `is_shadowed`, `intersect` + `prepare_computations`).
#include "rt_api_internal.hpp"

using namespace rtapi;

extern "C" {

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
  const bool batch = !stats && !(flags & RT_RENDER_EXHAUSTIVE) && fast_path(s) && per > 0;
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
      add_stats(sum, ds);
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

}  // extern "C"

namespace rtapi {
namespace {
// The row bands of a banded host render (render_banded):
// the frame's rows in nb <= 64 blocks of rb rows (one period of
// rt_render_block_pattern_device's mapping over the whole canvas), cut into
// `bands` contiguous runs of blocks. The first band takes band_pct of the rows,
// the others share the remainder in sizes falling by band_ratio percent per
// band. False: too few blocks to band.
struct BandPlan {
  int bands = 0;
  uint32_t rb = 0, nb = 0;
  uint32_t y0[kMaxBands + 1] = {};  // band k = rows [y0[k], y0[k + 1])
  uint64_t mask[kMaxBands] = {};    // band k's blocks
};
bool plan_bands(const rt_scene* s, uint32_t H, BandPlan& p) {
  p.bands = std::max(2, std::min(kMaxBands, s->tune.bands));
  p.rb = (H + 63) / 64;
  p.nb = (H + p.rb - 1) / p.rb;
  if (p.nb < (uint32_t)p.bands * 2) return false;
  const uint32_t nb = p.nb;
  const int bands = p.bands;
  uint32_t b[kMaxBands + 1] = {};
  b[1] = std::max<uint32_t>(1, std::min<uint32_t>(nb - (uint32_t)bands + 1, (uint32_t)((uint64_t)nb * s->tune.band_pct / 100)));
  double wsum = 0.0, wk = 1.0;
  for (int k = 1; k < bands; ++k, wk *= s->tune.band_ratio / 100.0) wsum += wk;
  double acc = 0.0;
  wk = 1.0;
  for (int k = 2; k < bands; ++k, wk *= s->tune.band_ratio / 100.0) {
    acc += wk;
    const uint32_t at = b[1] + (uint32_t)((nb - b[1]) * acc / wsum + 0.5);
    b[k] = std::min<uint32_t>(nb - (uint32_t)(bands - k), std::max<uint32_t>(b[k - 1] + 1, at));
  }
  b[bands] = nb;
  const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
  for (int k = 0; k <= bands; ++k) p.y0[k] = std::min(H, b[k] * p.rb);
  for (int k = 0; k < bands; ++k) {
    const uint64_t below_end = b[k + 1] >= 64 ? ~0ull : ((1ull << b[k + 1]) - 1ull);
    const uint64_t below_start = (1ull << b[k]) - 1ull;
    p.mask[k] = all & below_end & ~below_start;
  }
  return true;
}

// The band renders of one call: band k renders on its own stream (its own
// workspace, pinned to the call), starting when band k-1's render is done (or
// band_gen >= 0: when its generation band_gen has been launched), so the GPU
// works on one band at a time as in a whole-frame render while each band's
// copy to the host runs behind the later bands. Band k's
// rows go to d_out + y0[k] rows. On destruction every stream that received
// work drains first, then the workspaces are unpinned (under the scene's lock):
// no kernel or copy outlives the call.
struct BandRender {
  rt_scene* s;
  std::unique_lock<std::mutex>& lk;
  rt_scene::HostCtx* c;
  const BandPlan& p;
  hipStream_t st[kMaxBands] = {};
  rt_scene::WfSlot* used[kMaxBands] = {};
  int n_enq = 0;  // band streams with work enqueued
  BandRender(rt_scene* s_, std::unique_lock<std::mutex>& lk_, rt_scene::HostCtx* c_, const BandPlan& p_)
      : s(s_), lk(lk_), c(c_), p(p_) {}
  ~BandRender() {
    for (int k = 0; k < n_enq; ++k)
      if (hipStreamSynchronize(st[k]) != hipSuccess) (void)hipGetLastError();
    if (!lk.owns_lock()) lk.lock();
    for (int k = 0; k < p.bands; ++k) unpin(k);
  }
  BandRender(const BandRender&) = delete;
  BandRender& operator=(const BandRender&) = delete;
  void unpin(int k) {
    if (used[k]) {
      --used[k]->pins;
      used[k] = nullptr;
    }
  }
  int open() {
    st[0] = c->stream;
    for (int k = 1; k < p.bands; ++k) {
      if (!c->band_stream[k - 1]) RT_HIP(hipStreamCreateWithFlags(&c->band_stream[k - 1], hipStreamNonBlocking));
      st[k] = c->band_stream[k - 1];
    }
    for (int k = 0; k < p.bands; ++k)
      if (!c->band_ev[k]) RT_HIP(hipEventCreateWithFlags(&c->band_ev[k], hipEventDisableTiming));
    return RT_OK;
  }
  // enqueues band k's render (under the scene's lock)
  int render(int k, const DevCamera& dc, uint32_t W, uint32_t aa, uint32_t max_depth) {
    if (k > 0) RT_HIP(hipStreamWaitEvent(st[k], c->band_ev[k - 1], 0));  // band k after band k-1's render
    const uint32_t rows = p.y0[k + 1] - p.y0[k];
    const bool early = s->tune.band_gen >= 0 && k + 1 < p.bands;
    bool recorded = false;
    n_enq = k + 1;
    int rc = run_render(s, dc, nullptr, rows * W * aa, aa, max_depth, p.rb, 0, 1, c->d_out + (size_t)p.y0[k] * W * 3,
                        st[k], nullptr, nullptr, 0, &used[k], nullptr, 1, false, &lk, false, true, p.nb, p.mask[k],
                        early ? c->band_ev[k] : nullptr, s->tune.band_gen, &recorded, &s->band_sizing);
    if (rc != RT_OK) return rc;
    if (!recorded) RT_HIP(hipEventRecord(c->band_ev[k], st[k]));
    return RT_OK;
  }
  // every band stream drained (the scene's lock released meanwhile); the first error
  int wait_all() {
    lk.unlock();  // the workspaces stay pinned to this call
    hipError_t first = hipSuccess;
    for (int k = 0; k < n_enq; ++k) {
      const hipError_t e = hipStreamSynchronize(st[k]);
      if (e != hipSuccess && first == hipSuccess) first = e;
    }
    lk.lock();
    if (first != hipSuccess) return fail(RT_ERR_HIP, std::string("banded render: ") + hipGetErrorString(first));
    return RT_OK;
  }
  // after wait_all: band k's workspace read back (learned sizes, overflow) and unpinned
  int overflowed(int k, bool* over) {
    *over = false;
    if (!used[k]) return RT_OK;
    used[k]->wf->learn(s->band_sizing);
    RT_HIP(used[k]->wf->take_overflow(over));
    unpin(k);
    return RT_OK;
  }
};
}  // namespace

// `Camera::render` into a host canvas with the device-to-host copy overlapped
// (rt_render_ex): the bands of plan_bands, each band's copy to
// the host behind its render while the next bands render. Every pixel is that
// of the whole-frame render (a pattern only chooses which rows a render owns).
// The caller's canvas must be pinned (rt_host_buffer_alloc), registered by the
// caller (`host_ready`: rt_render_multi) or registrable for the call (d2h =
// 1); RT_ERR_NO_DEVICE asks the caller for the one-render path. A band that
// overflowed its arenas is rendered again, synchronously, before the call
// returns (every synchronous call returns a complete frame). On every return
// after the first band is enqueued, every band stream has drained first: no
// kernel or copy into the canvas outlives the call (its registration, its
// pinned workspaces, the caller's buffer).
int render_banded(rt_scene* s, std::unique_lock<std::mutex>& lk, rt_scene::HostCtx* c, const rt_camera_desc& cam,
                  uint32_t max_depth, uint32_t aa, double* out_rgb, bool host_ready) {
  const uint32_t W = cam.hsize, H = cam.vsize;
  BandPlan p;
  if (!plan_bands(s, H, p)) return RT_ERR_NO_DEVICE;
  const size_t bytes = (size_t)W * H * 3 * sizeof(double);
  bool registered = false;
  if (!host_ready && !pinned_block(out_rgb, bytes)) {
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
  BandRender br(s, lk, c, p);  // (after unreg: it drains its streams before the canvas is unregistered)
  int rc = br.open();
  if (rc != RT_OK) return rc;
  const DevCamera dc = to_dev_camera(cam);
  auto copy = [&](int k) -> int {
    const size_t off = (size_t)p.y0[k] * W * 3;
    RT_HIP(hipMemcpyAsync(out_rgb + off, c->d_out + off, (size_t)(p.y0[k + 1] - p.y0[k]) * W * 3 * sizeof(double),
                          hipMemcpyDeviceToHost, br.st[k]));
    return RT_OK;
  };
  for (int k = 0; k < p.bands; ++k) {
    if ((rc = br.render(k, dc, W, aa, max_depth)) != RT_OK) return rc;
    if ((rc = copy(k)) != RT_OK) return rc;
  }
  if ((rc = br.wait_all()) != RT_OK) return rc;
  for (int k = 0; k < p.bands; ++k) {
    bool over = false;
    if ((rc = br.overflowed(k, &over)) != RT_OK) return rc;
    if (!over) continue;
    // (its canvas rows are NaN: render the band again, synchronously, with the arenas grown)
    const uint32_t rows = p.y0[k + 1] - p.y0[k];
    rc = run_render(s, dc, nullptr, rows * W * aa, aa, max_depth, p.rb, 0, 1, c->d_out + (size_t)p.y0[k] * W * 3,
                    br.st[k], nullptr, nullptr, 0, nullptr, nullptr, 1, true, &lk, false, false, p.nb, p.mask[k],
                    nullptr, -1, nullptr, &s->band_sizing);
    if (rc != RT_OK) return rc;
    if ((rc = copy(k)) != RT_OK) return rc;
    lk.unlock();
    const hipError_t e = hipStreamSynchronize(br.st[k]);
    lk.lock();
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("banded render: ") + hipGetErrorString(e));
  }
  return RT_OK;
}

}  // namespace rtapi

extern "C" {

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
  if (!stats && flags == 0 && s->tune.bands > 1 && fast_path(s) && n_pix * aa_samples >= ((uint64_t)1 << 20)) {
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
    RT_HIP(hipMalloc(&c->d_ppm_rows, (size_t)H * 4 + ((size_t)H + 1) * 8 + 8));  // row lengths, row offsets
    c->ppm_rows_cap = H;
  }
  unsigned long long* d_off = (unsigned long long*)(((uintptr_t)c->d_ppm_rows + (size_t)H * 4 + 7) & ~(uintptr_t)7);
  if (!c->h_len) RT_HIP(hipHostMalloc((void**)&c->h_len, sizeof(unsigned long long), hipHostMallocDefault));
  struct Drain {  // no kernel or copy of this call outlives it (the context goes back to the pool)
    hipStream_t st;
    ~Drain() {
      if (hipStreamSynchronize(st) != hipSuccess) (void)hipGetLastError();
    }
  } drain{c->stream};
  DevStats ds{};
  float ms = 0.f;
  const DevCamera dc = to_dev_camera(*camera);
  const uint32_t n_tasks = (uint32_t)(n_pix * aa_samples);
  // The render, the encoder and the text's length in one pass of the stream: the host waits
  // once, then reads the workspace's overflow record; a frame that outgrew its arenas is
  // rendered again synchronously (with stats the render is synchronous anyway).
  rt_scene::WfSlot* used = nullptr;
  struct Unpin {
    rt_scene::WfSlot*& w;
    std::unique_lock<std::mutex>& lk;
    ~Unpin() {
      if (!w) return;
      if (!lk.owns_lock()) lk.lock();
      --w->pins;
    }
  } unpin{used, lk};
  rc = run_render(s, dc, nullptr, n_tasks, aa_samples, max_depth, H, 0, 1, c->d_out, c->stream, stats ? &ds : nullptr,
                  stats ? &ms : nullptr, 0, stats ? nullptr : &used, nullptr, 1, stats != nullptr, &lk, false,
                  stats == nullptr);
  if (rc != RT_OK) return rc;
  auto encode = [&]() -> int {
    RT_HIP(ppm_encode_device(c->d_out, W, H, c->d_ppm, c->ppm_cap, (unsigned*)c->d_ppm_rows, d_off, hd, c->stream));
    RT_HIP(hipMemcpyAsync(c->h_len, d_off + H, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    lk.unlock();
    const hipError_t e = hipStreamSynchronize(c->stream);
    lk.lock();
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("rt_render_ppm: ") + hipGetErrorString(e));
    return RT_OK;
  };
  if ((rc = encode()) != RT_OK) return rc;
  if (used) {
    used->wf->learn(s->sizing);
    bool over = false;
    RT_HIP(used->wf->take_overflow(&over));
    --used->pins;
    used = nullptr;
    if (over) {  // (the canvas was poisoned: render it again, growing the arenas until it fits)
      rc = run_render(s, dc, nullptr, n_tasks, aa_samples, max_depth, H, 0, 1, c->d_out, c->stream, nullptr, nullptr,
                      0, nullptr, nullptr, 1, true, &lk);
      if (rc != RT_OK) return rc;
      if ((rc = encode()) != RT_OK) return rc;
    }
  }
  const int d2h = s->tune.d2h;
  lk.unlock();
  *out_len = hd.n + (size_t)*c->h_len;
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

}  // extern "C"
