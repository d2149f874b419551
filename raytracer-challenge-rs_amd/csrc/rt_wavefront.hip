// rt_wavefront.hip — the wavefront render pipeline (see rt_wavefront.hpp).
//
// Why wavefront on MI355X: the work per ray is a brute-force loop over every
// shape (the reference's `World::intersect`), identical for every ray of a
// kind. Flat per-generation queues keep every lane of every wave busy (no
// recursion-tree tail), and the trace kernels are small loops with few live
// registers, so 8 waves per SIMD hide the ~20-cycle dependent f64 latency.
// Primary rays share the camera origin, so their object-space origin o' and
// c = o'.o' - 1 are computed once per sphere per frame (exactly the same
// operations, so bit-identical) and each primary sphere test drops from 28 to
// 16 f64 operations.
//
// This file: the host side (Wavefront: workspaces, arenas, the generation
// loop, launches). Device code: rt_wf_device.hpp (trace and fused kernels),
// rt_wf_combine.hip (frame init, combine, average), rt_wavefront_glb.hip (the
// launches over the global-memory images, their own code object).
#include "rt_wf_device.hpp"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstring>

#pragma clang fp contract(off)

namespace rtamd {

int wf_tuning_apply(WfTuning& t, const char* key, int value) {
  struct Knob {
    const char* name;
    int WfTuning::*field;
    int lo, hi;
  };
  static const Knob knobs[] = {
      {"accel", &WfTuning::accel, 0, 1},           {"skip_shadow", &WfTuning::skip_shadow, 0, 1},
      {"shadow_lb", &WfTuning::shadow_lb, 0, 1},   {"image", &WfTuning::image, 0, 3},
      {"treelet", &WfTuning::treelet, 0, 1},       {"treelet_deltas", &WfTuning::treelet_deltas, 0, 1},
      {"shadow_stream", &WfTuning::shadow_stream, 0, 2}, {"adaptive_block", &WfTuning::adaptive_block, 0, 1},
      {"prim_lane", &WfTuning::prim_lane, 0, 2},   {"arena_pct", &WfTuning::arena_pct, 1, 100},
      {"wide", &WfTuning::wide, 0, 1},
      {"lds_wide", &WfTuning::lds_wide, 0, 1},
      {"d2h", &WfTuning::d2h, 0, 1},               {"bands", &WfTuning::bands, 1, 4},
      {"band_pct", &WfTuning::band_pct, 5, 95},   {"band_gen", &WfTuning::band_gen, -1, 8},
      {"band_ratio", &WfTuning::band_ratio, 30, 100}, {"multi_gather", &WfTuning::multi_gather, 0, 1},
      {"own_sphere", &WfTuning::own_sphere, 0, 2}, {"spread", &WfTuning::spread, 0, 1}};
  if (!key) return 0;
  for (const Knob& k : knobs) {
    if (std::strcmp(key, k.name) != 0) continue;
    if (value < k.lo || value > k.hi || (k.field == &WfTuning::image && value == 2)) return -1;
    t.*(k.field) = value;
    return 1;
  }
  return 0;
}

// ---------------------------------------------------------- host side
// Per-launch profiling: while a kernel class is being timed (Wavefront::pmark)
// its launch carries the start/stop events in the dispatch itself
// (hipExtLaunchKernel, WF_LAUNCH), so no event packets sit between the kernels
// and a profiled frame runs like an unprofiled one.
static thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
static thread_local int t_ev_used = 0;

Wavefront::~Wavefront() {
  for (auto& g : gens_) {
    (void)hipFree(g.rays); (void)hipFree(g.hits); (void)hipFree(g.nodes); (void)hipFree(g.colors);
    (void)hipFree(g.shadow_nodes); (void)hipFree(g.geo); (void)hipFree(g.surf);
  }
  (void)hipFree(colors_); (void)hipFree(parents_); (void)hipFree(rays_[0]); (void)hipFree(rays_[1]);
  if (d_gtab_) (void)hipFree(d_gtab_);
  if (d_gsh_) (void)hipFree(d_gsh_);
  if (d_cnt_) (void)hipFree(d_cnt_);
  if (d_shard_) (void)hipFree(d_shard_);
  if (d_prim_) (void)hipFree(d_prim_);
  if (d_frames_) (void)hipFree(d_frames_);
  if (h_rec_) (void)hipHostFree(h_rec_);
  if (ev0_) (void)hipEventDestroy(ev0_);
  if (ev1_) (void)hipEventDestroy(ev1_);
  for (hipEvent_t e : fork_ev_)
    if (e) (void)hipEventDestroy(e);
  if (join_ev_) (void)hipEventDestroy(join_ev_);
  if (side_) (void)hipStreamDestroy(side_);
  for (hipEvent_t e : pev_) (void)hipEventDestroy(e);
}

hipError_t Wavefront::pmark(hipStream_t s, int cls, bool begin) {
  (void)s;
  if (!profiling_ || !(pmask_ & (1 << cls))) return hipSuccess;
  if (begin) {
    const size_t idx = 2 * pn_;
    while (pev_.size() <= idx + 1) {
      hipEvent_t e;
      WF_CHECK(hipEventCreate(&e));
      pev_.push_back(e);
    }
    if (pcls_.size() <= pn_) pcls_.resize(pn_ + 1);
    pcls_[pn_] = cls;
    t_ev_start = pev_[idx];
    t_ev_stop = pev_[idx + 1];
    t_ev_used = 0;
  } else {
    t_ev_start = t_ev_stop = nullptr;
    if (t_ev_used != 1) return hipErrorInvalidValue;  // a timed class is exactly one launch
    ++pn_;
  }
  return hipSuccess;
}

hipError_t Wavefront::last_profile(WfProfile* out) {
  *out = WfProfile{};
  for (size_t i = 0; i < pn_; ++i) {
    WF_CHECK(hipEventSynchronize(pev_[2 * i + 1]));
    float ms = 0.f;
    WF_CHECK(hipEventElapsedTime(&ms, pev_[2 * i], pev_[2 * i + 1]));
    out->ms[pcls_[i]] += ms;
  }
  if (pframes_ > 1)
    for (int c = 0; c < WF_NCLASS; ++c) out->ms[c] /= (double)pframes_;
  WfCounters hc{};
  if (d_cnt_) WF_CHECK(hipMemcpy(&hc, d_cnt_, sizeof hc, hipMemcpyDeviceToHost));  // nothing rendered yet: zeros
  for (int c = 0; c < 3; ++c) {
    out->rays[c] = prof_rays_[c];
    out->disc[c] = (double)hc.disc(c);
    out->tests[c] = (double)hc.tests(c);
    out->boxes[c] = (double)hc.boxes(c);
  }
  if (last_fused_) {  // the fast path's generations sized themselves: their rays from the record (any stream, 0 too)
    std::vector<unsigned> rays;
    WF_CHECK(last_counts(rays));
    out->rays[WF_PRIMARY] = rays.empty() ? 0.0 : (double)rays[0];
    double sec = 0.0;
    for (size_t g = 1; g < rays.size(); ++g) sec += (double)rays[g];
    out->rays[WF_CLOSEST] = sec;
  }
  for (int c = 0; c < 2; ++c) {
    out->sh_rays[c] = (double)hc.sh_rays(c);
    out->sh_tests[c] = (double)hc.sh_tests(c);
  }
  if (last_fused_) out->rays[WF_SHADOW] = out->sh_rays[0] + out->sh_rays[1];  // traced inside the fused launches
  out->bvh = last_bvh_ ? 1 : 0;
  out->fused = last_fused_ ? 1 : 0;
  return hipSuccess;
}

// Grow-only per-generation buffers of the exhaustive pipeline (12.5 %
// headroom on each reallocation): the rays, colours, hits, nodes, hit
// geometry, lighting terms (slots x n_lights) and the shadow list.
template <typename T>
static hipError_t grow(T*& p, size_t& cap, size_t need) {
  need = std::max<size_t>(need, 1);
  if (cap >= need) return hipSuccess;
  (void)hipFree(p);
  p = nullptr;
  cap = 0;
  const size_t n = need + need / 8;
  WF_CHECK(hipMalloc(&p, n * sizeof(T)));
  cap = n;
  return hipSuccess;
}
hipError_t Wavefront::ensure_gen(size_t g, size_t slots, size_t n_lights, size_t list_slots) {
  if (gens_.size() <= g) gens_.resize(g + 1);
  WfGenBuf& b = gens_[g];
  WF_CHECK(grow(b.rays, b.cap_rays, slots));
  WF_CHECK(grow(b.colors, b.cap_colors, slots * 3));
  WF_CHECK(grow(b.hits, b.cap_hits, slots));
  WF_CHECK(grow(b.nodes, b.cap_nodes, slots));
  WF_CHECK(grow(b.geo, b.cap_geo, slots));
  WF_CHECK(grow(b.surf, b.cap_surf, slots * std::max<size_t>(n_lights, 1) * 3));
  WF_CHECK(grow(b.shadow_nodes, b.cap_list, list_slots));
  return hipSuccess;
}

// The fast path's arenas (device-sized generations): colour slots, parent
// records, and ray slots per ping-pong buffer. Grow-only (12.5 % headroom),
// unless `exact` (the arena_pct test hook), which reallocates to the size
// asked for.
hipError_t Wavefront::ensure_arenas(unsigned long long colors, unsigned long long parents, unsigned long long rays,
                                    bool exact) {
  auto fit = [&](auto*& p, unsigned long long& cap, unsigned long long need, size_t elem, int n_bufs) -> hipError_t {
    need = std::max<unsigned long long>(need, 1);
    if (exact ? cap == need : cap >= need) return hipSuccess;
    const unsigned long long n = exact ? need : need + need / 8;
    for (int k = 0; k < n_bufs; ++k) {
      (void)hipFree((&p)[k]);
      (&p)[k] = nullptr;
    }
    cap = 0;
    for (int k = 0; k < n_bufs; ++k) WF_CHECK(hipMalloc((void**)&(&p)[k], n * elem));
    cap = n;
    return hipSuccess;
  };
  WF_CHECK(fit(colors_, color_cap_, colors, 3 * sizeof(double), 1));
  WF_CHECK(fit(parents_, par_cap_, parents, sizeof(ParentRec), 1));
  WF_CHECK(fit(rays_[0], ray_cap_, rays, sizeof(WfRay), 2));
  return hipSuccess;
}

hipError_t Wavefront::take_overflow(bool* was) {
  *was = false;
  if (!h_rec_) return hipSuccess;
  volatile WfHostRec* r = h_rec_;
  if (!r->overflow) return hipSuccess;
  *was = true;
  const unsigned long long nc = r->need_colors, np = r->need_parents, nr = r->need_rays;
  r->overflow = 0;
  // at least double whatever fell short: the generations after the overflowing
  // one never ran, so their needs are unknown
  auto next = [](unsigned long long cap, unsigned long long need) {
    return need > cap ? std::max(need + need / 4, 2 * cap) : cap;
  };
  return ensure_arenas(next(color_cap_, nc), next(par_cap_, np), next(ray_cap_, nr), false);
}

void Wavefront::learn(WfSizing& sz) const {
  if (!h_rec_) return;
  const volatile WfHostRec* r = h_rec_;
  if (r->frames == 0) return;
  const unsigned n0 = r->n_real, ng = std::min<unsigned>((unsigned)r->n_gens, (unsigned)kMaxGen);
  if (n0 == 0 || ng == 0) return;
  double sum = 0.0, mx = 0.0;
  for (unsigned g = 0; g < ng; ++g) {
    const double c = (double)r->counts[g];
    if (g + 1 < ng) sum += c;  // the last generation spawns no children
    mx = std::max(mx, c);
  }
  sz.rho = std::max(sz.rho, sum / n0);
  sz.mu = std::max(sz.mu, mx / n0);
}

hipError_t Wavefront::last_counts(std::vector<unsigned>& rays) {
  rays.clear();
  if (!lr_.fused) {
    rays = lr_.rays;
    return hipSuccess;
  }
  WF_CHECK(hipStreamSynchronize(lr_.stream));
  const volatile WfHostRec* r = h_rec_;
  const unsigned ng = std::min<unsigned>((unsigned)r->n_gens, (unsigned)kMaxGen);
  for (unsigned g = 0; g < ng; ++g) rays.push_back((unsigned)r->counts[g]);
  while (rays.size() > 1 && rays.back() == 0) rays.pop_back();
  return hipSuccess;
}

// The shadow stream of the current device (recreated if the device changed).
hipError_t Wavefront::ensure_side() {
  int dev = 0;
  WF_CHECK(hipGetDevice(&dev));
  if (side_ && side_dev_ == dev) return hipSuccess;
  if (side_) {
    WF_CHECK(hipStreamSynchronize(side_));
    (void)hipStreamDestroy(side_);
    for (hipEvent_t& e : fork_ev_)
      if (e) { (void)hipEventDestroy(e); e = nullptr; }
    if (join_ev_) { (void)hipEventDestroy(join_ev_); join_ev_ = nullptr; }
    side_ = nullptr;
  }
  WF_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  for (hipEvent_t& e : fork_ev_) WF_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  WF_CHECK(hipEventCreateWithFlags(&join_ev_, hipEventDisableTiming));
  side_dev_ = dev;
  return hipSuccess;
}

hipError_t Wavefront::ensure_misc(size_t n_diag, unsigned n_frames) {
  if (!d_cnt_) WF_CHECK(hipMalloc(&d_cnt_, sizeof(WfCounters)));
  if (!h_rec_) {
    WF_CHECK(hipHostMalloc((void**)&h_rec_, sizeof(WfHostRec), hipHostMallocMapped));
    std::memset((void*)h_rec_, 0, sizeof(WfHostRec));
    WF_CHECK(hipHostGetDevicePointer((void**)&d_rec_, h_rec_, 0));
  }
  if (!d_gtab_) WF_CHECK(hipMalloc(&d_gtab_, (kMaxGen + 1) * sizeof(WfGenTab)));
  if (!d_gsh_) WF_CHECK(hipMalloc(&d_gsh_, kMaxGen * sizeof(unsigned)));
  if (!d_shard_) WF_CHECK(hipMalloc(&d_shard_, (size_t)kMaxGen * 2 * kShards * kShardStride * sizeof(unsigned)));
  if (!ev0_) WF_CHECK(hipEventCreate(&ev0_));
  if (!ev1_) WF_CHECK(hipEventCreate(&ev1_));
  if (n_frames > 1 && !d_frames_) WF_CHECK(hipMalloc(&d_frames_, sizeof(FrameTable)));
  const size_t np = (n_diag + 4) * n_frames;  // one set of primary records per frame of a batch
  if (prim_cap_ < np) {
    if (d_prim_) (void)hipFree(d_prim_);
    d_prim_ = nullptr;
    WF_CHECK(hipMalloc(&d_prim_, np * sizeof(PrimRec)));
    prim_cap_ = np;
  }
  return hipSuccess;
}

template <typename K>
static int occupancy_grid(K kern, int block, size_t lds, unsigned n) {
  int dev = 0, n_cu = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  long long want = ((long long)n + block - 1) / block;
  long long cap = (long long)n_cu * per_cu;
  long long g = std::min(want, cap);
  return (int)std::max(g, 1LL);
}

static constexpr size_t kWfLdsLimit = kFusedLdsLimit;
static_assert(kFusedBlockThreads == kTraceBlock, "rt_api.cpp sizes the pair image with kFusedBlockThreads");

// Threads per block of a trace launch over n rays. A trace block holds one CU
// (its LDS image), so a launch of fewer than (CUs x kTraceBlock) rays would
// leave CUs idle with full-size blocks: such launches spread their rays over
// every CU instead, in blocks of a multiple of 64 threads (small shards of a
// multi-GPU frame, the deep generations). The kernels index their LDS stacks
// with the kTraceBlock stride and loop over gridDim x blockDim, so any block
// size up to kTraceBlock gives the same results.
// (WfTuning::adaptive_block; frames in flight fill idle CUs better without it)
static int trace_block(unsigned n, int adaptive) {
  if (!adaptive) return kTraceBlock;
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (n_cu < 1) n_cu = 1;
  }
  const unsigned per = ((n + (unsigned)n_cu - 1) / (unsigned)n_cu + 63u) & ~63u;
  return (int)std::min<unsigned>(std::max<unsigned>(per, 64u), (unsigned)kTraceBlock);
}

// Per-launch profiling: see t_ev_start.
#define WF_LAUNCH(kern, grid, block, lds, stream, ...)                                                  \
  do {                                                                                                 \
    if (t_ev_start) {                                                                                  \
      hipExtLaunchKernelGGL(kern, grid, block, lds, stream, t_ev_start, t_ev_stop, 0, __VA_ARGS__);    \
      ++t_ev_used;                                                                                     \
    } else {                                                                                           \
      hipLaunchKernelGGL(kern, grid, block, lds, stream, __VA_ARGS__);                                 \
    }                                                                                                  \
  } while (0)

template <typename K>
static hipError_t launch_lds(K kern, size_t lds, unsigned n, hipStream_t stream, const DevScene& sc,
                             const DevCamera& cam, const WfArgs& a, int block) {
  if (lds > 0) WF_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  WF_LAUNCH(kern, dim3(occupancy_grid(kern, block, lds, n)), dim3(block), lds, stream, sc, cam, a);
  return hipGetLastError();
}

// ---- the exhaustive pipeline (counted launches: the reference's every-shape loop)
template <bool QUADS>
static hipError_t launch_closest_exh(const DevScene& sc, const DevCamera& cam, const WfArgs& a, bool primary,
                                     bool lds_ok, unsigned n, hipStream_t stream, const WfTuning& tn) {
  const int tb = trace_block(n, tn.adaptive_block);
  if (primary)
    return launch_lds(wf_trace_closest<true, true, QUADS, 8>, wf_lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes, true),
                      n, stream, sc, cam, a, tb);
  if (lds_ok)
    return launch_lds(wf_trace_closest<true, false, QUADS, 8>, wf_lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes, false),
                      n, stream, sc, cam, a, tb);
  return launch_lds(wf_trace_closest<false, false, QUADS, 8>, 0, n, stream, sc, cam, a, tb);
}
template <bool QUADS>
static hipError_t launch_shadow_exh(const DevScene& sc, const WfArgs& a, bool lds_ok, hipStream_t stream,
                                    const WfTuning& tn) {
  const int tb = trace_block(a.n_shadow, tn.adaptive_block);
  if (lds_ok) {
    const size_t lds = wf_lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes, false);
    auto k = wf_trace_shadow<true, QUADS, 8>;
    WF_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    WF_LAUNCH(k, dim3(occupancy_grid(k, tb, lds, a.n_shadow)), dim3(tb), lds, stream, sc, a);
  } else {
    auto k = wf_trace_shadow<false, QUADS, 8>;
    WF_LAUNCH(k, dim3(occupancy_grid(k, tb, 0, a.n_shadow)), dim3(tb), 0, stream, sc, a);
  }
  return hipGetLastError();
}

// the global-memory images' launches live in their own code object (rt_wavefront_glb.o)
static hipError_t launch_global(int lane, bool quads, bool tally, bool cam_rays, const DevScene& sc,
                                const DevCamera& cam, const WfArgs& a, size_t dyn, unsigned n, hipStream_t stream,
                                int block) {
  const hipError_t e =
      wf_launch_global(lane, quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, t_ev_start, t_ev_stop);
  if (t_ev_start) ++t_ev_used;
  return e;
}

// ---- the fast path: one fused launch per generation (image choice: see lane_scene)
template <bool QUADS, bool TALLY>
static hipError_t launch_fused_q(const DevScene& sc, const DevCamera& cam, WfArgs a, bool primary, unsigned n,
                                 hipStream_t stream, const WfTuning& tn) {
  // (spread: the whole grid, whatever n; the kernel deals the chunks over every block)
  if (a.spread && !tn.adaptive_block) n = 1u << 30;
  const int tb = trace_block(n, tn.adaptive_block);
  const size_t dl = a.use_lb ? delta_lds_bytes(sc) : 0;
  size_t dyn = 0;
  a.lds_flags = 0;
  // primary rays: the wave traversal, or with prim_lane the per-lane walk of the pair image or of
  // the four-wide hierarchy (the launches below, reading camera rays)
  const bool wide_ok = tn.image != 1 && tn.wide && sc.bvhw16 && wide_stack_bytes(sc) <= kWfLdsLimit / 2;
  // prim_lane 1 (default): any per-lane image (C3 primary class 0.128 -> 0.125 ms/frame with the LDS
  // four-wide image; C5's global image: 2.06 -> 2.16 ms with binary32 nodes in round 4, 2.17 -> 2.01
  // ms with the binary16 ones, round 6); 2: the LDS images only
  const bool wide_lds = sc.bvhw && tn.lds_wide && wide_lds_bytes(sc) + dl <= kWfLdsLimit;
  const bool lds_img = tn.image == 0 && (pair_lds_bytes(sc) <= kWfLdsLimit || wide_lds);
  const bool lane_prim = tn.prim_lane == 1 ? (lds_img || wide_ok) : tn.prim_lane == 2 ? lds_img : false;
  if (primary && !lane_prim) {
    const size_t room = kWfLdsLimit - (size_t)(kTraceBlock / 64) * (kBvhMaxDepth + 4) * 4;
    if (sph_lds_bytes(sc) <= room) { a.lds_flags |= kLdsSpheres; dyn += sph_lds_bytes(sc); }
    if (dl && dyn + dl <= room) { a.lds_flags |= kLdsDeltas; dyn += dl; }
    return launch_lds(wf_trace_fused<true, QUADS, 0, TALLY>, dyn, n, stream, sc, cam, a, tb);
  }
  const bool cam_rays = a.g == 0 && a.camera_mode;  // only generation 0 of a camera render reads camera rays
  if (tn.image == 0 && wide_lds) {
    // the four-wide hierarchy and the 48-B sphere records in LDS, with the light buffer's distances
    dyn = wide_lds_bytes(sc);
    if (dl) { a.lds_flags |= kLdsDeltas; dyn += dl; }
    return cam_rays ? launch_lds(wf_trace_fused<false, QUADS, 15, TALLY, true>, dyn, n, stream, sc, cam, a, tb)
                    : launch_lds(wf_trace_fused<false, QUADS, 15, TALLY, false>, dyn, n, stream, sc, cam, a, tb);
  }
  if (tn.image == 0 && pair_lds_bytes(sc) <= kWfLdsLimit) {
    // the pair layout in LDS (scenes whose four-wide image does not fit beside the distances);
    // the light buffer's distances take what room is left
    dyn = pair_lds_bytes(sc);
    if (dl && dyn + dl <= kWfLdsLimit) {
      a.lds_flags |= kLdsDeltas;
      dyn += dl;
    }
    return cam_rays ? launch_lds(wf_trace_fused<false, QUADS, 14, TALLY, true>, dyn, n, stream, sc, cam, a, tb)
                    : launch_lds(wf_trace_fused<false, QUADS, 14, TALLY, false>, dyn, n, stream, sc, cam, a, tb);
  }
  if (wide_ok) {
    // the four-wide hierarchy: its 16-bit stack, then the light buffer's distances
    // and/or a treelet of its top nodes in the room left
    const size_t room = kWfLdsLimit - wide_stack_bytes(sc);
    dyn = wide_stack_bytes(sc);
    if (dl && dl <= room && (!tn.treelet || tn.treelet_deltas)) { a.lds_flags |= kLdsDeltas; dyn += dl; }
    if (tn.treelet) {
      a.n_top = (unsigned)std::min<size_t>((size_t)sc.n_bvhw, (kWfLdsLimit - dyn) / sizeof(BvhWide16));
      dyn += (size_t)a.n_top * sizeof(BvhWide16);
    }
    return launch_global(4, QUADS, TALLY, cam_rays, sc, cam, a, dyn, n, stream, tb);
  }
  if (tn.image != 1 && sc.bvh_depth <= kLaneLdsDepth) {
    const size_t room = kWfLdsLimit - (size_t)kLaneLdsDepth * kTraceBlock * 4;
    // the room left beside the stack: the light buffer's distances and/or a treelet
    const bool deltas = dl && dl <= room && (!tn.treelet || tn.treelet_deltas);
    if (deltas) { a.lds_flags |= kLdsDeltas; dyn = dl; }
    if (tn.treelet) {
      a.n_top = (unsigned)std::min<size_t>((size_t)sc.n_bvh, (room - dyn) / sizeof(BvhNode));
      dyn += (size_t)a.n_top * sizeof(BvhNode);
    }
    return launch_global(3, QUADS, TALLY, cam_rays, sc, cam, a, dyn, n, stream, tb);
  }
  if (dl && dl <= kWfLdsLimit) { a.lds_flags |= kLdsDeltas; dyn = dl; }
  return launch_global(1, QUADS, TALLY, cam_rays, sc, cam, a, dyn, n, stream, tb);
}
static hipError_t launch_fused(const DevScene& sc, const DevCamera& cam, const WfArgs& a, bool primary, unsigned n,
                               hipStream_t stream, bool tally, const WfTuning& tn) {
  // QUADS: solids outside the hierarchies, or the hierarchy over the other records
  const bool quads = sc.n_fx_quads > 0 || sc.n_obvh > 0 || sc.n_lbvh > 0;
  if (tally)
    return quads ? launch_fused_q<true, true>(sc, cam, a, primary, n, stream, tn)
                 : launch_fused_q<false, true>(sc, cam, a, primary, n, stream, tn);
  return quads ? launch_fused_q<true, false>(sc, cam, a, primary, n, stream, tn)
               : launch_fused_q<false, false>(sc, cam, a, primary, n, stream, tn);
}

hipError_t Wavefront::render(const DevScene& sc, const DevCamera& cam, bool camera_mode, const double* d_in_rays,
                             unsigned n0, unsigned aa, unsigned max_depth, unsigned row_block, unsigned shard,
                             unsigned n_shards, double* d_out, hipStream_t stream, WfSizing& sz, DevStats* stats,
                             float* ms_kernel, const WfTuning& tn, bool solo, unsigned flags,
                             const FrameTable* batch, unsigned n_frames, unsigned blk_period,
                             unsigned long long blk_mask) {
  if (max_depth + 2 > (unsigned)kMaxGen) return hipErrorInvalidValue;
  if (blk_period > 64 || (blk_period && (blk_mask == 0 || (blk_period < 64 && (blk_mask >> blk_period) != 0))))
    return hipErrorInvalidValue;
  blk_period_ = blk_period;
  blk_mask_ = blk_period ? blk_mask : 0ull;
  if (aa == 0 || aa > 16 || (aa & (aa - 1)) != 0 || (!camera_mode && aa != 1) || n0 % aa != 0)
    return hipErrorInvalidValue;
  if (n_frames == 0 || n_frames > kMaxFrames || (n_frames > 1 && !batch)) return hipErrorInvalidValue;
  WF_CHECK(ensure_misc((size_t)sc.n_diag, n_frames));
  // BVH traversal (fused generations) and skipped shadow rays unless the
  // reference's every-shape loop is asked for; counting (stats) never changes the algorithm
  const bool exhaustive = (flags & WF_EXHAUSTIVE) != 0;
  const bool count = stats != nullptr || (flags & WF_COUNT) != 0;
  const bool bvh = tn.accel != 0 && !exhaustive && (sc.n_bvh > 0 || sc.n_obvh > 0 || sc.n_lbvh > 0);
  const bool fused = bvh;
  // (a counted render of a scene with groups traces every shadow ray: the reference's shape
  // tests then come from the group gates each ray met, GateSkips)
  const bool skip_shadow = !exhaustive && tn.skip_shadow != 0 && !(count && sc.n_groups > 0);
  // a batch of frames: the fast path's generations over every frame's root
  // rays (uncounted camera renders only; the caller renders others one by one)
  const unsigned frame_real = n0;
  if (n_frames > 1) {
    if (!camera_mode || !fused || count || n0 == 0) return hipErrorInvalidValue;
    n0 = n_frames * ((n0 + 63u) & ~63u);
  }
  const bool use_prim = camera_mode && sc.n_diag > 0 &&
                        (fused || wf_lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes, true) <= kWfLdsLimit);
  {  // counters zeroed, generation 0 placed and the primary records written by one launch
    static_assert(sizeof(WfCounters) % 16 == 0, "WfCounters is zeroed in 16-B words");
    const unsigned n_a = (unsigned)(sizeof(WfCounters) / 16);
    const unsigned n_b = (unsigned)((size_t)(max_depth + 2) * 2 * kShards * kShardStride * sizeof(unsigned) / 16);
    const unsigned work = std::max<unsigned>(std::max(n_a, n_b), use_prim ? n_frames * ((unsigned)sc.n_diag + 4) : 0u);
    const FrameTable none{};
    WF_LAUNCH(wf_frame_init, dim3(std::min<unsigned>((work + 255) / 256, 256u)), dim3(256), 0, stream, sc, cam,
              d_prim_, use_prim ? 1u : 0u, (uint4*)d_cnt_, n_a, (uint4*)d_shard_, n_b, n_frames > 1 ? *batch : none,
              d_frames_, n_frames, fused ? d_gtab_ : (WfGenTab*)nullptr);
    WF_CHECK(hipGetLastError());
  }
  const bool timed = ms_kernel != nullptr || (flags & WF_TIME) != 0;
  if (timed) WF_CHECK(hipEventRecord(ev0_, stream));
  if (profiling_) pframes_ += n_frames;  // class times are reported per frame
  prof_rays_[0] = prof_rays_[1] = prof_rays_[2] = 0;
  last_bvh_ = bvh;
  last_fused_ = fused;
  lr_.stream = stream;
  lr_.fused = fused;
  if (fused)
    WF_CHECK(render_fast(sc, cam, camera_mode, d_in_rays, n0, frame_real, aa, max_depth, row_block, shard, n_shards,
                         d_out, stream, sz, count, skip_shadow, tn, batch, n_frames));
  else
    WF_CHECK(render_exhaustive(sc, cam, camera_mode, d_in_rays, n0, aa, max_depth, row_block, shard, n_shards, d_out,
                               stream, count, skip_shadow, tn, solo));
  if (timed) WF_CHECK(hipEventRecord(ev1_, stream));
  lr_.L = (unsigned)sc.n_lights; lr_.n0 = n0; lr_.max_depth = max_depth;
  lr_.counted = count; lr_.exact_disc = !bvh && !skip_shadow; lr_.bvh = bvh;
  lr_.n_diag = (unsigned long long)sc.n_diag; lr_.n_gen = (unsigned long long)sc.n_gen;
  lr_.n_planes = (unsigned long long)sc.n_planes; lr_.n_quads = (unsigned long long)sc.n_quads;
  if (stats || ms_kernel) {
    WF_CHECK(hipStreamSynchronize(stream));
    if (ms_kernel) WF_CHECK(hipEventElapsedTime(ms_kernel, ev0_, ev1_));
  }
  if (stats) WF_CHECK(read_stats(stats));
  return hipSuccess;
}

// Slots of generation g+1 that generation g's launch reserves for n_g rays
// (bind_generation: 64 regions of 128 `per`), and of its parent list.
static unsigned long long gen_slots(unsigned long long n) {
  const unsigned long long groups = ((n + 63) / 64 + kShardGroup - 1) / kShardGroup;
  return (unsigned long long)kShards * 128ull * kShardGroup * ((groups + kShards - 1) / kShards);
}

// The fast path (DESIGN.md "Device-sized generations"): every launch of the
// frame is enqueued at once; each generation's launch finds its own ray count
// on the device. The host only sizes the arenas, from the scene's learned
// ratios (WfSizing) or, when smaller, from the exact bound of the recursion
// (every ray spawning `branch` children); a frame that outgrows them is
// reported through the workspace's overflow record (take_overflow).
hipError_t Wavefront::render_fast(const DevScene& sc, const DevCamera& cam, bool camera_mode, const double* d_in_rays,
                                  unsigned n0, unsigned frame_real, unsigned aa, unsigned max_depth,
                                  unsigned row_block, unsigned shard, unsigned n_shards, double* d_out,
                                  hipStream_t stream, WfSizing& sz, bool count, bool skip_shadow, const WfTuning& tn,
                                  const FrameTable* batch, unsigned n_frames) {
  const bool averaged = aa > 1;
  const unsigned n_real = frame_real * n_frames;
  // ---- arena sizes
  learn(sz);  // this workspace's last recorded frame (a frame still in flight may be stale: a hint only)
  const unsigned D = max_depth;
  double c_bound = (double)n0, p_bound = 0.0, r_bound = camera_mode ? 0.0 : (double)n0;
  {
    double ng = (double)n0;
    for (unsigned g = 0; g < D; ++g) {
      const double s = (double)gen_slots((unsigned long long)std::min(ng, 4.0e9));
      c_bound += s;
      p_bound += s / 2.0;
      r_bound = std::max(r_bound, s);
      ng = std::min(ng * (double)sz.branch, 4.0e9);
      if (ng == 0.0) break;
    }
  }
  const double rho = sz.rho > 0.0 ? sz.rho : 8.0, mu = sz.mu > 0.0 ? sz.mu : 2.0;
  const double min_region = (double)gen_slots(1);  // one wave-iteration's regions: 64 x 128 x kShardGroup
  const double c_learn = (double)n0 + 2.5 * rho * n_real + min_region * D;
  const double p_learn = 1.25 * rho * n_real + min_region / 2.0 * D;
  const double r_learn = std::max(camera_mode ? 0.0 : (double)n0, 2.5 * mu * n_real + min_region);
  double want_c = std::min(c_bound, c_learn), want_p = std::min(p_bound, p_learn), want_r = std::min(r_bound, r_learn);
  // the test hook shrinks the arenas once per setting (the re-renders after an
  // overflow then grow them as usual)
  const bool squeeze = tn.arena_pct < 100 && tn.arena_pct != squeezed_pct_;
  squeezed_pct_ = tn.arena_pct;
  if (squeeze) {
    want_c = std::max((double)n0, want_c * tn.arena_pct / 100.0);
    want_p *= tn.arena_pct / 100.0;
    want_r = std::max(camera_mode ? 0.0 : (double)n0, want_r * tn.arena_pct / 100.0);
  }
  hipError_t ea = ensure_arenas((unsigned long long)want_c, (unsigned long long)want_p, (unsigned long long)want_r,
                                squeeze);
  // Sizes guessed before the scene has learned any frame (rho, mu) can exceed what the
  // device holds (a large canvas, branch 2, deep recursion): halve them down to the
  // smallest useful arenas. A frame that outgrows them overflows: a synchronous call
  // renders it again with the arenas grown, an asynchronous one is poisoned (NaN) and
  // reported (poison_frames, rt_scene_check).
  const double floor_c = (double)n0 + min_region * D, floor_p = min_region / 2.0 * D;
  const double floor_r = std::max(camera_mode ? 0.0 : (double)n0, min_region);
  for (int k = 0; ea == hipErrorOutOfMemory && k < 16 && (want_c > floor_c || want_p > floor_p || want_r > floor_r);
       ++k) {
    (void)hipGetLastError();
    want_c = std::max(floor_c, want_c / 2.0);
    want_p = std::max(floor_p, want_p / 2.0);
    want_r = std::max(floor_r, want_r / 2.0);
    ea = ensure_arenas((unsigned long long)want_c, (unsigned long long)want_p, (unsigned long long)want_r, true);
  }
  WF_CHECK(ea);
  if (!camera_mode)  // batch rays: n0 x 6 doubles -> generation 0's ray buffer
    WF_CHECK(hipMemcpy2DAsync(rays_[0], sizeof(WfRay), d_in_rays, 6 * sizeof(double), 6 * sizeof(double), n0,
                              hipMemcpyDeviceToDevice, stream));
  WfArgs a{};
  a.dev_sized = 1;
  a.colors_direct = averaged ? 0u : 1u;
  a.gtab = d_gtab_;
  a.gsh = d_gsh_;
  a.ray_buf[0] = rays_[0];
  a.ray_buf[1] = rays_[1];
  a.color_base = colors_;
  a.par_base = parents_;
  a.color_cap = color_cap_;
  a.par_cap = par_cap_;
  a.ray_cap = ray_cap_;
  a.hrec = d_rec_;
  a.aa = aa;
  a.rows = frame_real / aa / (cam.hsize ? cam.hsize : 1);
  a.n_frames = n_frames; a.frame_rays = n0 / n_frames; a.frame_real = frame_real; a.frames = d_frames_;
  a.cnt = d_cnt_;
  a.prim = d_prim_;
  a.max_depth = max_depth;
  a.camera_mode = camera_mode ? 1u : 0u;
  a.row_block = row_block; a.shard = shard; a.n_shards = n_shards;
  a.blk_period = blk_period_; a.blk_mask = blk_mask_;
  a.skip_shadow = skip_shadow ? 1u : 0u;
  a.own_sphere = sc.obj_diag ? (unsigned)tn.own_sphere : 0u;
  a.spread = tn.spread ? 1u : 0u;
  a.count = count ? 1u : 0u;
  a.use_lb = (tn.shadow_lb && sc.lb_cells) ? 1u : 0u;
  const bool use_prim = camera_mode && sc.n_diag > 0;
  // an upper bound on any generation's rays, for the grid of the device-sized
  // launches (the kernels stride over what they find)
  const unsigned kAnyRays = 1u << 30;
  for (unsigned g = 0; g <= max_depth; ++g) {
    a.g = g;
    a.colors = d_out;  // generation 0 without AA: the output (bind_generation keeps it)
    a.n = g == 0 ? n0 : 0u;
    a.in_cnt = g == 0 ? nullptr : shard_cnt(g, 0);
    a.out_cnt = shard_cnt(g + 1, 0);
    a.sh_cnt = shard_cnt(g, 1);
    const bool prim_launch = g == 0 && use_prim;
    const int ccls = prim_launch ? WF_PRIMARY : WF_CLOSEST;
    a.disc_slot = (unsigned)ccls;
    if (g == 0) prof_rays_[ccls] += n_real;
    WF_CHECK(pmark(stream, ccls, true));
    WF_CHECK(launch_fused(sc, cam, a, prim_launch, g == 0 ? n0 : kAnyRays, stream, count, tn));
    WF_CHECK(pmark(stream, ccls, false));
    if (gen_ev_ && (int)g == gen_ev_g_) {
      WF_CHECK(hipEventRecord(gen_ev_, stream));
      gen_ev_done_ = true;
    }
  }
  gen_ev_ = nullptr;
  // combine, deepest generation first (only the nodes with children; the last
  // generation has none). Generation 0's pass records the frame's counts.
  static int combine_grid = 0;
  if (combine_grid == 0) combine_grid = occupancy_grid(wf_combine_parents, kWfBlock, 0, kAnyRays);
  for (int g = max_depth > 0 ? (int)max_depth - 1 : 0; g >= 0; --g) {
    a.g = (unsigned)g;
    a.colors = d_out;
    a.sh_cnt = shard_cnt((unsigned)g, 1);
    a.out_cnt = shard_cnt(1, 0);
    WF_CHECK(pmark(stream, WF_COMBINE, true));
    WF_LAUNCH(wf_combine_parents, dim3(combine_grid), dim3(kWfBlock), 0, stream, sc, cam, a);
    WF_CHECK(hipGetLastError());
    WF_CHECK(pmark(stream, WF_COMBINE, false));
  }
  if (averaged) {
    const unsigned n_pix = n_frames * (frame_real / aa);
    WF_CHECK(pmark(stream, WF_COMBINE, true));
    WfArgs v{};
    v.aa = aa; v.rows = frame_real / aa / cam.hsize;
    v.n_frames = n_frames; v.frame_rays = n0 / n_frames; v.frame_real = frame_real; v.frames = d_frames_;
    v.cnt = d_cnt_;
    WF_LAUNCH(wf_average, dim3(occupancy_grid(wf_average, kWfBlock, 0, n_pix)), dim3(kWfBlock), 0, stream, v,
              cam.hsize, colors_, n_pix, d_out);
    WF_CHECK(hipGetLastError());
    WF_CHECK(pmark(stream, WF_COMBINE, false));
  }
  (void)batch;
  lr_.last = max_depth;
  lr_.rays.clear();
  lr_.shadows.clear();
  return hipSuccess;
}

// The exhaustive pipeline (the reference's every-shape loop, counted renders):
// each generation's ray and shadow-ray counts are read back before the next
// launch (synchronous); its buffers are per generation.
hipError_t Wavefront::render_exhaustive(const DevScene& sc, const DevCamera& cam, bool camera_mode,
                                        const double* d_in_rays, unsigned n0, unsigned aa, unsigned max_depth,
                                        unsigned row_block, unsigned shard, unsigned n_shards, double* d_out,
                                        hipStream_t stream, bool count, bool skip_shadow, const WfTuning& tn,
                                        bool solo) {
  const bool averaged = aa > 1;
  const unsigned L = (unsigned)sc.n_lights;
  std::vector<unsigned> rays(max_depth + 2, 0), shadows(max_depth + 2, 0);
  rays[0] = n0;
  WF_CHECK(ensure_gen(0, n0, L, 0));
  if (!camera_mode) {
    // batch rays: n0 x 6 doubles -> WfRay queue of generation 0
    WF_CHECK(hipMemcpy2DAsync(gens_[0].rays, sizeof(WfRay), d_in_rays, 6 * sizeof(double), 6 * sizeof(double), n0,
                              hipMemcpyDeviceToDevice, stream));
  }
  const bool prim_lds = wf_lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes, true) <= kWfLdsLimit;
  const bool gen_lds = wf_lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes, false) <= kWfLdsLimit;
  const bool use_prim = camera_mode && prim_lds && sc.n_diag > 0;
  // Shadow traces of generation g depend only on closest(g), like closest(g+1);
  // they run on the side stream, forked after closest(g) and joined before the
  // combine pass (DESIGN.md "Shadow stream").
  hipStream_t sh_stream = stream;
  if (tn.shadow_stream == 2 || (tn.shadow_stream == 1 && solo)) {
    WF_CHECK(ensure_side());
    sh_stream = side_;
  }
  bool forked = false;
  unsigned last = 0;
  // per-region capacity of each generation's sharded arrays (generation 0 is
  // dense) and of its shadow list
  std::vector<unsigned> caps(max_depth + 2, 0), list_caps(max_depth + 2, 0);
  for (unsigned g = 0; g <= max_depth; ++g) {
    const unsigned n = rays[g];
    if (n == 0) break;
    last = g;
    // wave-iteration q of this generation appends its shadow rays to region
    // (q / kShardGroup) mod kShards, at most `per` wave-iterations of <= 64 L
    // shadow rays each; its reflected and refracted rays to region (q / kShardGroup)
    // mod (kShards / 2) of their half, at most 2 `per` wave-iterations of <= 64 rays
    // each (shard_append)
    const unsigned groups = ((n + 63) / 64 + kShardGroup - 1) / kShardGroup;
    const unsigned per = kShardGroup * ((groups + kShards - 1) / kShards);
    const unsigned out_cap = g < max_depth ? 128u * per : 0u, sh_cap = 64u * L * per;
    caps[g + 1] = out_cap;
    list_caps[g] = sh_cap;
    WF_CHECK(ensure_gen(g, g == 0 ? n : (size_t)kShards * caps[g], L, (size_t)kShards * sh_cap));
    WF_CHECK(ensure_gen(g + 1, (size_t)kShards * out_cap, L, 0));
    WfArgs a{};
    WfGenBuf& B = gens_[g];
    a.rays = B.rays; a.hits = B.hits; a.nodes = B.nodes; a.shadow_nodes = B.shadow_nodes;
    a.geo = B.geo; a.surf = B.surf;
    a.colors = (g == 0 && !averaged) ? d_out : B.colors;
    a.aa = aa;
    a.rows = n0 / aa / (cam.hsize ? cam.hsize : 1);
    a.n_frames = 1; a.frame_rays = n0; a.frame_real = n0;
    a.next_rays = gens_[g + 1].rays;
    a.child_colors = gens_[g + 1].colors;
    a.cnt = d_cnt_;
    a.prim = d_prim_;
    a.n = n;
    a.in_cnt = g == 0 ? nullptr : shard_cnt(g, 0);
    a.in_cap = caps[g];
    a.out_cnt = shard_cnt(g + 1, 0);
    a.out_cap = out_cap;
    a.sh_cnt = shard_cnt(g, 1);
    a.sh_cap = sh_cap;
    a.g = g; a.max_depth = max_depth;
    a.camera_mode = camera_mode ? 1u : 0u;
    a.row_block = row_block; a.shard = shard; a.n_shards = n_shards;
    a.blk_period = blk_period_; a.blk_mask = blk_mask_;
    a.skip_shadow = skip_shadow ? 1u : 0u;
    a.count = count ? 1u : 0u;
    // 1. closest hit
    const bool prim_launch = g == 0 && use_prim;
    const int ccls = prim_launch ? WF_PRIMARY : WF_CLOSEST;
    a.disc_slot = (unsigned)ccls;
    prof_rays_[ccls] += n;
    WF_CHECK(pmark(stream, ccls, true));
    if (sc.n_quads > 0) WF_CHECK(launch_closest_exh<true>(sc, cam, a, prim_launch, gen_lds, n, stream, tn));
    else WF_CHECK(launch_closest_exh<false>(sc, cam, a, prim_launch, gen_lds, n, stream, tn));
    WF_CHECK(pmark(stream, ccls, false));
    // 2. prepare_computations + spawn
    WF_CHECK(pmark(stream, WF_PREP, true));
    WF_LAUNCH(wf_prep, dim3(occupancy_grid(wf_prep, kWfBlock, 0, n)), dim3(kWfBlock), 0, stream, sc, cam, a);
    WF_CHECK(hipGetLastError());
    WF_CHECK(pmark(stream, WF_PREP, false));
    {  // the next generation's size and this one's shadow list, read back
      std::vector<unsigned> hr((size_t)kShards * kShardStride), hs(hr.size());
      WF_CHECK(hipMemcpyAsync(hr.data(), shard_cnt(g + 1, 0), hr.size() * sizeof(unsigned), hipMemcpyDeviceToHost,
                              stream));
      WF_CHECK(hipMemcpyAsync(hs.data(), shard_cnt(g, 1), hs.size() * sizeof(unsigned), hipMemcpyDeviceToHost, stream));
      WF_CHECK(hipStreamSynchronize(stream));
      unsigned nr = 0, ns = 0;
      for (int k = 0; k < kShards; ++k) {
        nr += hr[(size_t)k * kShardStride] + hr[(size_t)k * kShardStride + 1];  // front + back (shard_append)
        ns += hs[(size_t)k * kShardStride];
      }
      rays[g + 1] = g < max_depth ? nr : 0;
      shadows[g] = ns;
    }
    a.n_shadow = shadows[g];
    // 3. shadow rays
    if (a.n_shadow) {
      a.disc_slot = WF_SHADOW;
      prof_rays_[WF_SHADOW] += a.n_shadow;
      if (sh_stream != stream) {
        WF_CHECK(hipEventRecord(fork_ev_[g], stream));
        WF_CHECK(hipStreamWaitEvent(sh_stream, fork_ev_[g], 0));
        forked = true;
      }
      WF_CHECK(pmark(sh_stream, WF_SHADOW, true));
      if (sc.n_quads > 0) WF_CHECK(launch_shadow_exh<true>(sc, a, gen_lds, sh_stream, tn));
      else WF_CHECK(launch_shadow_exh<false>(sc, a, gen_lds, sh_stream, tn));
      WF_CHECK(pmark(sh_stream, WF_SHADOW, false));
    }
    if (count) {
      WF_LAUNCH(wf_count_kinds, dim3(occupancy_grid(wf_count_kinds, 256, 0, n)), dim3(256), 0, stream, a);
      WF_CHECK(hipGetLastError());
    }
  }
  if (forked) {  // join: the combine pass reads every generation's lighting terms
    WF_CHECK(hipEventRecord(join_ev_, sh_stream));
    WF_CHECK(hipStreamWaitEvent(stream, join_ev_, 0));
  }
  // 4. combine, deepest generation first
  for (int g = (int)last; g >= 0; --g) {
    WfArgs a{};
    WfGenBuf& B = gens_[g];
    a.rays = B.rays; a.nodes = B.nodes; a.surf = B.surf;
    a.colors = (g == 0 && !averaged) ? d_out : B.colors;
    a.aa = aa;
    a.rows = n0 / aa / (cam.hsize ? cam.hsize : 1);
    a.n_frames = 1; a.frame_rays = n0; a.frame_real = n0;
    a.child_colors = gens_[g + 1].colors;
    a.n = rays[g];
    a.in_cnt = g == 0 ? nullptr : shard_cnt((unsigned)g, 0);
    a.in_cap = caps[g];
    a.g = (unsigned)g; a.max_depth = max_depth;
    a.camera_mode = camera_mode ? 1u : 0u;
    a.row_block = row_block; a.shard = shard; a.n_shards = n_shards;
    a.blk_period = blk_period_; a.blk_mask = blk_mask_;
    if (a.n == 0) continue;
    WF_CHECK(pmark(stream, WF_COMBINE, true));
    WF_LAUNCH(wf_combine, dim3(occupancy_grid(wf_combine, kWfBlock, 0, a.n)), dim3(kWfBlock), 0, stream, sc, cam, a);
    WF_CHECK(hipGetLastError());
    WF_CHECK(pmark(stream, WF_COMBINE, false));
  }
  if (averaged) {
    const unsigned n_pix = n0 / aa;
    WF_CHECK(pmark(stream, WF_COMBINE, true));
    WfArgs a{};
    a.aa = aa; a.rows = n0 / aa / cam.hsize;
    a.n_frames = 1; a.frame_rays = n0; a.frame_real = n0;
    WF_LAUNCH(wf_average, dim3(occupancy_grid(wf_average, kWfBlock, 0, n_pix)), dim3(kWfBlock), 0, stream, a,
              cam.hsize, gens_[0].colors, n_pix, d_out);
    WF_CHECK(hipGetLastError());
    WF_CHECK(pmark(stream, WF_COMBINE, false));
  }
  lr_.rays = rays;
  lr_.shadows = shadows;
  lr_.last = last;
  return hipSuccess;
}

hipError_t Wavefront::read_stats(DevStats* out) {
  *out = DevStats{};
  if (!lr_.counted || !d_cnt_) return hipErrorInvalidValue;
  WF_CHECK(hipStreamSynchronize(lr_.stream));
  WfCounters hc;
  WF_CHECK(hipMemcpy(&hc, d_cnt_, sizeof hc, hipMemcpyDeviceToHost));
  std::vector<unsigned> counts;
  WF_CHECK(last_counts(counts));
  DevStats s{};
  unsigned long long rays = 0, hits = 0, traced_shadows = 0;
  for (unsigned g = 0; g < counts.size() && g < (unsigned)kMaxGen; ++g) {
    rays += counts[g];
    if (!lr_.fused && g < lr_.shadows.size()) traced_shadows += lr_.shadows[g];
    hits += hc.n_hit[g];
    s.rays_reflect += hc.n_refl[g];
    s.rays_refract += hc.n_refr[g];
  }
  if (lr_.fused) traced_shadows = hc.sh_rays(0) + hc.sh_rays(1);
  // the reference's work: every hit runs is_shadowed once per light (world.rs:41-56), and
  // World::intersect tests every shape for every ray (world.rs:31-38)
  const unsigned long long shadows = hits * (unsigned long long)lr_.L;
  s.rays_primary = lr_.n0;
  s.rays_shadow = shadows;
  // (minus the shapes whose group's box a ray missed: Group::intersect never calls them)
  s.sphere_tests = (rays + shadows) * (lr_.n_diag + lr_.n_gen) - hc.gated(0);
  s.plane_tests = (rays + shadows) * lr_.n_planes - hc.gated(1);
  s.other_tests = (rays + shadows) * lr_.n_quads - hc.gated(2);
  s.sphere_disc_ge0 = lr_.exact_disc ? hc.disc(0) + hc.disc(1) + hc.disc(2) : ~0ull;
  s.exhaustive = lr_.exact_disc ? 1u : 0u;
  // what the kernels did
  s.rays_shadow_traced = traced_shadows;
  const unsigned long long traced = rays + traced_shadows;
  s.sphere_tests_executed = (lr_.bvh ? hc.tests(0) + hc.tests(1) + hc.tests(2) + traced * lr_.n_gen
                                     : traced * (lr_.n_diag + lr_.n_gen)) - hc.gated(0);
  s.box_tests_executed = hc.boxes(0) + hc.boxes(1) + hc.boxes(2);
  *out = s;
  return hipSuccess;
}

}  // namespace rtamd
