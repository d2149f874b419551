// rt_api.cpp — the C-ABI's small entry points (include/rt_render.h): errors,
// ABI sizes, pinned host buffers, `Matrix::inverse` and `Camera::new` on the
// host, rt_scene_check, and the development hooks (per-class profiling,
// tuning knobs, plain streams). Scene creation is rt_scene.cpp, the renders
// rt_render.cpp, multi-GPU rt_multi.cpp (rt_api_internal.hpp lists them).
#include "rt_api_internal.hpp"
#include "rt_pow.hpp"

namespace rtapi {

thread_local std::string g_err;
int g_bvh_leaf = 0;     // BVH leaf size at scene creation (tuning knob "bvh_leaf"); 0 = automatic: 2, or 1 when
                        // the LDS image cannot hold the scene (C5: 1024² frame 4.42 -> 4.31 ms; C3 best at 2)
int g_bvh_ct = 70;      // SAH node-visit cost in percent of a sphere test (tuning knob "bvh_ct")
// light-buffer cells per cube-map face edge at scene creation ("lb_res"): 0 = none, -1 = by
// scene size (256, or 512 above 4096 diagonal spheres: C5 47.1 -> 46.7 ms/frame, C3 unchanged)
int g_lb_res = -1;
std::mutex g_tune_mu;
WfTuning g_tune_defaults;

namespace {
// Pinned host buffers (rt_host_buffer_alloc): page-locked blocks the DMA
// engine writes at the full link rate, kept in a small pool on release so a
// frame loop's canvases reuse the same pages (no registration, no page faults).
// The pool is never torn down (the HIP runtime may be gone at process exit).
std::mutex g_pin_mu;
std::vector<std::pair<void*, size_t>> g_pin_live, g_pin_free;
size_t g_pin_free_bytes = 0;
constexpr size_t kPinPoolBytes = (size_t)1 << 30;
}  // namespace

bool pinned_block(const void* p, size_t n) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  for (const auto& b : g_pin_live)
    if ((const char*)p >= (const char*)b.first && (const char*)p + n <= (const char*)b.first + b.second) return true;
  return false;
}

}  // namespace rtapi

using namespace rtapi;

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

// Rays of each generation of the scene's last render (dev tool): returns the
// number of generations written into out[0 .. max).
int rtamd_wf_gen_counts(const rt_scene* cs, unsigned* out, int max) {
  if (!cs || !out || max < 0) return fail(RT_ERR_INVALID_ARGUMENT, "null scene or output");
  rt_scene* s = const_cast<rt_scene*>(cs);
  std::lock_guard<std::mutex> lk(s->mu);
  if (!s->last_wf) return 0;
  RT_DEVICE(s->device);
  std::vector<unsigned> rays;
  RT_HIP(s->last_wf->wf->gen_counts(rays));
  const int n = std::min<int>((int)rays.size(), max);
  for (int i = 0; i < n; ++i) out[i] = rays[(size_t)i];
  return n;
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
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess || !p) {
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

uint32_t rt_shard_rows(uint32_t vsize, uint32_t row_block, uint32_t shard, uint32_t n_shards) {
  if (row_block == 0 || n_shards == 0 || shard >= n_shards) return 0;
  uint32_t rows = 0;
  for (uint32_t blk = shard; (uint64_t)blk * row_block < vsize; blk += n_shards) {
    uint32_t y0 = blk * row_block;
    rows += std::min(row_block, vsize - y0);
  }
  return rows;
}

uint32_t rt_pattern_rows(uint32_t vsize, uint32_t row_block, uint32_t period, uint64_t mask) {
  if (row_block == 0 || !valid_pattern(period, mask)) return 0;
  uint32_t rows = 0;
  for (uint64_t blk = 0; blk * row_block < vsize; ++blk)
    if ((mask >> (blk % period)) & 1u) rows += std::min<uint32_t>(row_block, vsize - (uint32_t)(blk * row_block));
  return rows;
}

// Development/test hooks (not in the public ABI): the specular term's pow
// (rt_pow.hpp, glibc 2.35's algorithm) for n pairs, on the host (the same
// source compiled for the CPU; tests/test_pow.py) and on the device (device
// buffers, stream-ordered then synchronised; tests/test_gpu_pow.py).
void rtamd_pow_host(const double* x, const double* y, size_t n, double* out) {
  for (size_t i = 0; i < n; ++i) out[i] = rtamd::pow_glibc(x[i], y[i]);
}
int rtamd_pow_device(const double* d_x, const double* d_y, size_t n, double* d_out, void* stream) {
  return guarded([&]() -> int {
  if (n >= (1ull << 31)) return fail(RT_ERR_INVALID_ARGUMENT, "batch too large");
  RT_HIP(launch_pow(d_x, d_y, (int)n, d_out, (hipStream_t)stream));
  RT_HIP(hipStreamSynchronize((hipStream_t)stream));
  return RT_OK;
  });
}

}  // extern "C"
