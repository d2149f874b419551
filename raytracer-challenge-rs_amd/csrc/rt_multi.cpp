// rt_multi.cpp — `Camera::render_multithreaded` across devices
// (camera.rs:150-217) and the RCCL hooks of the multi-process assembler.
//
// rt_render_multi returns a HOST canvas, like the reference's owned Canvas.
// Every device renders its interleaved row blocks (the reference's row-block
// partition, camera.rs:157-172, interleaved so sky and dense rows spread
// evenly) and its own DMA engine copies them straight into the canvas rows it
// owns, over its own link: a host canvas needs no gather, and no device
// funnels the frame through one link. Each device is driven by its own host
// thread (the call enqueues, waits and checks overflows per device in
// parallel); the one-device call is rt_render's banded path (row bands, each
// band's copy behind the next band's render). The RCCL form (every shard
// gathered into device 0 with one grouped ncclGather, then copied out of
// device 0) is kept behind the scene knob `multi_gather` (a test hook: it
// runs the same grouped gather on one device through a single-rank
// communicator).
#include "rt_api_internal.hpp"

using namespace rtapi;

namespace {

// A host canvas registered for every device (portable) for the duration of the
// calls that write it. Calls writing one canvas at once (rt_render_multi's
// workers, or concurrent part renders) share one registration: the first
// registers, the last one out unregisters, so no registration ends while
// another call's copies still land in the pages.
struct HostReg {
  void* p = nullptr;
  bool ready = false;  // pinned or registered: the DMA engines write it directly
  bool owned = false;
  HostReg(void* ptr, size_t bytes, int device) : p(ptr) {
    if (pinned_block(ptr, bytes)) {
      ready = true;
      return;
    }
    std::lock_guard<std::mutex> lk(mu());
    for (Entry& e : table())
      if (e.p == ptr && e.bytes == bytes) {
        ++e.refs;
        ready = owned = true;
        return;
      }
    DeviceGuard dg(device);
    if (hipHostRegister(ptr, bytes, hipHostRegisterPortable) != hipSuccess) {
      (void)hipGetLastError();
      // (memory the caller pinned or registered itself is written directly too)
      hipPointerAttribute_t at{};
      ready = hipPointerGetAttributes(&at, ptr) == hipSuccess && at.type == hipMemoryTypeHost;
      (void)hipGetLastError();
      return;
    }
    table().push_back(Entry{ptr, bytes, 1});
    ready = owned = true;
  }
  ~HostReg() {
    if (!owned) return;
    std::lock_guard<std::mutex> lk(mu());
    auto& t = table();
    for (size_t i = 0; i < t.size(); ++i)
      if (t[i].p == p && --t[i].refs == 0) {
        if (hipHostUnregister(p) != hipSuccess) (void)hipGetLastError();
        t.erase(t.begin() + (long)i);
        return;
      }
  }
  HostReg(const HostReg&) = delete;
  HostReg& operator=(const HostReg&) = delete;

 private:
  struct Entry {
    void* p;
    size_t bytes;
    int refs;
  };
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::vector<Entry>& table() {
    static std::vector<Entry> t;
    return t;
  }
};

// One device's rows of the canvas: shard `shard` of `n_shards` (blocks of
// `row_block` rows, block b on shard b mod n_shards), rendered on the scene's
// device into a device buffer of its rows, then copied into the canvas rows
// it owns: one 2-D copy for its full blocks (n_shards * row_block rows apart
// in the canvas), one more for a short last block. `host_ready`: the canvas is
// pinned or registered for every device. Synchronous; an overflowed render is
// rendered again inside run_render.
int render_shard_to_host(rt_scene* s, const rt_camera_desc& cam, uint32_t max_depth, uint32_t aa,
                         uint32_t row_block, uint32_t shard, uint32_t n_shards, double* out_rgb, bool host_ready,
                         DevStats* ds, float* ms) {
  std::unique_lock<std::mutex> lk(s->mu);
  RT_DEVICE(s->device);
  const uint32_t W = cam.hsize, H = cam.vsize;
  const uint32_t rows = rt_shard_rows(H, row_block, shard, n_shards);
  if (rows == 0) return RT_OK;
  CtxLease cx{s, lk};
  RT_TAKE_CTX(cx);
  rt_scene::HostCtx* c = cx.c;
  const uint64_t n_pix = (uint64_t)W * H;
  if (n_shards == 1 && !ds && s->tune.bands > 1 && fast_path(s) && n_pix * aa >= ((uint64_t)1 << 20)) {
    int rc = ensure_dev_buffer(&c->d_out, &c->out_cap, n_pix * 3);
    if (rc != RT_OK) return rc;
    rc = render_banded(s, lk, c, cam, max_depth, aa, out_rgb, host_ready);
    if (rc != RT_ERR_NO_DEVICE) return rc;  // (not bandable: render it whole below)
  }
  int rc = ensure_dev_buffer(&c->d_out, &c->out_cap, (size_t)rows * W * 3);
  if (rc != RT_OK) return rc;
  rc = run_render(s, to_dev_camera(cam), nullptr, rows * W * aa, aa, max_depth, row_block, shard, n_shards, c->d_out,
                  c->stream, ds, ms, 0, nullptr, nullptr, 1, true, &lk);
  if (rc != RT_OK) return rc;
  lk.unlock();  // the context is this call's
  if (!host_ready)  // (a canvas the DMA engine cannot write: the staged copy of rt_render, rows in shard order)
    return n_shards == 1 ? copy_to_host(c, s->tune.d2h, out_rgb, c->d_out, (size_t)rows * W * 3 * sizeof(double),
                                        c->stream)
                         : fail(RT_ERR_INVALID_ARGUMENT, "rt_render_multi: the canvas is neither pinned nor registrable");
  struct Drain {  // no copy into the caller's canvas outlives the call
    hipStream_t st;
    ~Drain() {
      if (hipStreamSynchronize(st) != hipSuccess) (void)hipGetLastError();
    }
  } drain{c->stream};
  const size_t row_bytes = (size_t)W * 3 * sizeof(double);
  if (n_shards == 1) {
    RT_HIP(hipMemcpyAsync(out_rgb, c->d_out, (size_t)rows * row_bytes, hipMemcpyDeviceToHost, c->stream));
  } else {
    uint32_t n_full = 0;  // this shard's full blocks (they come before a short last block)
    for (uint64_t blk = shard; (blk + 1) * row_block <= H; blk += n_shards) ++n_full;
    if (n_full)
      RT_HIP(hipMemcpy2DAsync(out_rgb + (size_t)shard * row_block * W * 3, (size_t)n_shards * row_block * row_bytes,
                              c->d_out, (size_t)row_block * row_bytes, (size_t)row_block * row_bytes, n_full,
                              hipMemcpyDeviceToHost, c->stream));
    const uint32_t last = H / row_block;  // a short last block, if this shard owns it
    if (H % row_block && last % n_shards == shard)
      RT_HIP(hipMemcpyAsync(out_rgb + (size_t)last * row_block * W * 3, c->d_out + (size_t)n_full * row_block * W * 3,
                            (size_t)(H % row_block) * row_bytes, hipMemcpyDeviceToHost, c->stream));
  }
  RT_HIP(hipStreamSynchronize(c->stream));
  return RT_OK;
}

// The RCCL form (scene knob multi_gather): every shard gathered into device 0
// (one grouped ncclGather), then each row block copied from device 0 into the
// canvas. The communicators and device buffers are cached on scenes[0] across
// calls (rt_scene::MultiCache) and rebuilt only when the scene set changes.
int render_multi_gather(rt_scene* const* scenes, int n_devices, const rt_camera_desc* camera, uint32_t max_depth,
                        uint32_t aa_samples, uint32_t row_block, double* out_rgb, rt_stats* stats) {
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
    {  // (one device too: the single-rank communicator runs the same grouped gather)
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
  // every stream this call enqueued on drains before any return (the canvas is the caller's)
  struct Drain {
    rt_scene* const* sc;
    int n;
    ~Drain() {
      for (int i = 0; i < n; ++i)
        if (hipSetDevice(i) == hipSuccess && hipStreamSynchronize(sc[i]->stream) != hipSuccess) (void)hipGetLastError();
    }
  } drain{scenes, n_devices};
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
  {
    if (ncclGroupStart() != ncclSuccess) return fail(RT_ERR_RCCL, "ncclGroupStart");
    for (int i = 0; i < n_devices; ++i)
      if (ncclGather(mc.send[i], i == 0 ? mc.recv : nullptr, per, ncclDouble, 0, mc.comms[i], scenes[i]->stream) !=
          ncclSuccess) {
        (void)ncclGroupEnd();
        return fail(RT_ERR_RCCL, "ncclGather");
      }
    if (ncclGroupEnd() != ncclSuccess) return fail(RT_ERR_RCCL, "ncclGroupEnd");
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
      stats->sphere_disc_ge0 = x.exhaustive ? stats->sphere_disc_ge0 + x.sphere_disc_ge0 : x.sphere_disc_ge0;
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
}

}  // namespace

extern "C" {

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
  const uint32_t W = camera->hsize, H = camera->vsize;
  uint32_t max_rows = 0;
  for (int i = 0; i < n_devices; ++i) max_rows = std::max(max_rows, rt_shard_rows(H, row_block, i, n_devices));
  if ((uint64_t)max_rows * W * aa_samples >= (1ull << 31))
    return fail(RT_ERR_INVALID_ARGUMENT, "shard too large for one launch");
  int gather = 0;
  {
    std::lock_guard<std::mutex> lk(scenes[0]->mu);
    gather = scenes[0]->tune.multi_gather;
  }
  DeviceGuard restore;  // the caller's device (the workers select theirs)
  if (gather) return render_multi_gather(scenes, n_devices, camera, max_depth, aa_samples, row_block, out_rgb, stats);
  const auto t0 = std::chrono::steady_clock::now();
  // The canvas, registered once for every device (portable) unless it is a pinned
  // block already; unregistered after every device's copies have completed
  // (the workers are joined before `reg` goes out of scope).
  const HostReg reg(out_rgb, (size_t)W * H * 3 * sizeof(double), scenes[0]->device);
  const bool host_ready = reg.ready;
  struct Shard {
    int rc = RT_OK;
    std::string err;
    DevStats ds{};
    float ms = 0.f;
  };
  std::vector<Shard> res((size_t)n_devices);
  auto work = [&](int i) {
    Shard& r = res[(size_t)i];
    r.rc = guarded([&]() -> int {
      return render_shard_to_host(scenes[i], *camera, max_depth, aa_samples, row_block, (uint32_t)i,
                                  (uint32_t)n_devices, out_rgb, host_ready, stats ? &r.ds : nullptr,
                                  stats ? &r.ms : nullptr);
    });
    if (r.rc != RT_OK) r.err = g_err;  // (this thread's message)
  };
  // one host thread per device (device 0 on the calling thread): each enqueues its
  // render and copies, waits for them and checks its arenas without waiting on the others
  std::vector<std::thread> pool;
  int spawned = 1;
  try {
    for (; spawned < n_devices; ++spawned) pool.emplace_back(work, spawned);
  } catch (...) {  // a thread that cannot start: that device runs on this thread below
  }
  work(0);
  for (int i = spawned; i < n_devices; ++i) work(i);
  for (std::thread& th : pool) th.join();
  for (int i = 0; i < n_devices; ++i)
    if (res[(size_t)i].rc != RT_OK) return fail(res[(size_t)i].rc, "device " + std::to_string(i) + ": " + res[(size_t)i].err);
  if (stats) {
    DevStats sum{};
    float ms = 0.f;  // ms_kernel: the slowest device's shard render
    for (const Shard& r : res) {
      add_stats(sum, r.ds);
      ms = std::max(ms, r.ms);
    }
    fill_stats(stats, sum, ms, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
  return RT_OK;
  });
}

// Development/test hook (not in the public ABI): one device's part of
// rt_render_multi on one scene: shard `shard` of `n_shards` rendered and copied
// into the rows it owns of a full-size host canvas. Lets one GPU run every
// device's part (tests/test_gpu_multi.py, tools/multi_probe.py).
int rtamd_render_shard_host(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth,
                            uint32_t aa_samples, uint32_t row_block, uint32_t shard, uint32_t n_shards,
                            double* out_rgb, rt_stats* stats) {
  return guarded([&]() -> int {
  if (!scene || !camera || !out_rgb) return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  if (row_block == 0 || n_shards == 0 || shard >= n_shards)
    return fail(RT_ERR_INVALID_ARGUMENT, "bad shard specification");
  if (camera->hsize == 0 || camera->vsize == 0) return fail(RT_ERR_INVALID_ARGUMENT, "empty camera");
  if (!valid_aa(aa_samples)) return fail(RT_ERR_INVALID_ARGUMENT, "aa_samples must be 1, 2, 4, 8 or 16");
  rt_scene* s = const_cast<rt_scene*>(scene);
  const auto t0 = std::chrono::steady_clock::now();
  const HostReg reg(out_rgb, (size_t)camera->hsize * camera->vsize * 3 * sizeof(double), s->device);
  DevStats ds{};
  float ms = 0.f;
  const int rc = render_shard_to_host(s, *camera, max_depth, aa_samples, row_block, shard, n_shards, out_rgb,
                                      reg.ready, stats ? &ds : nullptr, stats ? &ms : nullptr);
  if (rc == RT_OK && stats)
    fill_stats(stats, ds, ms, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  return rc;
  });
}

}  // extern "C"
