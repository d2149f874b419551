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
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstring>

#include "rt_device.hpp"
#include "rt_trace.hpp"
#include "rt_wavefront.hpp"

#pragma clang fp contract(off)

namespace rtamd {

[[maybe_unused]] constexpr int kWfBlock = 256;  // prep / shadow / combine

#ifndef RT_WF_GLOBAL_TU  // (the global-image TU: kernels and their launcher only)
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
      {"band_ratio", &WfTuning::band_ratio, 30, 100}};
  if (!key) return 0;
  for (const Knob& k : knobs) {
    if (std::strcmp(key, k.name) != 0) continue;
    if (value < k.lo || value > k.hi || (k.field == &WfTuning::image && value == 2)) return -1;
    t.*(k.field) = value;
    return 1;
  }
  return 0;
}
#endif

#define WF_CHECK(x)                        \
  do {                                     \
    hipError_t _e = (x);                   \
    if (_e != hipSuccess) return _e;       \
  } while (0)


// The calling wave's row of the work counters (WfCounters): lane 0 adds the
// wave's totals there.
__device__ __forceinline__ WfWorkRow* work_row(WfCounters* c) {
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  return c->work + (w & (kWorkRows - 1));
}

// Wave-aggregated queue append: every active lane calls it (convergent);
// lanes with want=true get consecutive slots (in lane order) of `per` entries.
__device__ __forceinline__ unsigned wave_append(unsigned* counter, bool want, unsigned per) {
  const unsigned long long m = __ballot(want);
  if (m == 0) return 0;
  const int leader = __ffsll((long long)m) - 1;
  unsigned base = 0;
  if ((int)lane_id() == leader) base = atomicAdd(counter, (unsigned)__popcll(m) * per);
  base = __shfl(base, leader, 64);
  const unsigned rank = (unsigned)__popcll(m & ((1ull << lane_id()) - 1ull));
  return base + rank * per;
}



// Queue appends without block barriers or hot counters (DESIGN.md "Sharded
// queues"). The queues of a generation are split into kShards regions of a
// fixed capacity; wave-iteration q (rays 64q .. 64q+63 of the generation)
// appends with one atomic per queue on a region's own counter (128 B apart),
// and groups of kShardGroup adjacent wave-iterations share a region, so
// neighbouring rays stay neighbours. Every lane of the wave calls it. A lane
// gets `n_s` consecutive parent-list (shadow-list) slots and one ray slot each
// for want_r / want_f (absolute slots; ~0u when a region is full, which the
// capacities rule out).
//
// The parent list: region (q / kShardGroup) mod kShards.
// The next generation's rays are sorted into four classes so that its waves
// hold rays of one class each (coherent traversal and shading):
//   reflected rays, cat_r = 0 / 1, and refracted rays, cat_f = 0 / 1 (the
//   caller's categories: reflections off planes or not; refractions leaving an
//   object or entering one).
// Reflected rays use the first half of the regions, refracted rays the second:
// region (q / kShardGroup) mod (kShards / 2) of the half. Category 0 fills a
// region from its front (counter word 0), category 1 from its back (counter
// word 1, slots cap-1, cap-2, ...). The capacity bound is that of one queue per
// region: a region takes at most 2 `per` wave-iterations (twice the
// wave-iterations of a kShards mapping) of at most 64 rays of its kind each
// (one per lane, whatever the category), i.e. 128 `per` = out_cap, front and
// back together. The reader sees 2 kShards virtual regions (shard_prefix<true>).
// C5 58.7 -> 51.3 ms/frame, C3 0.852 -> 0.83 ms (kinds, then categories).
__device__ __forceinline__ void shard_append(const WfArgs& a, unsigned q, unsigned n_s, bool want_r, bool want_f,
                                             unsigned& so, unsigned& ro, unsigned& fo, bool cat_r, bool cat_f) {
  const unsigned lane = lane_id();
  const unsigned s = (q / kShardGroup) % kShards;
  const unsigned p_r = (q / kShardGroup) % (kShards / 2), p_f = kShards / 2 + p_r;
  const unsigned long long mr0 = __ballot(want_r && !cat_r), mr1 = __ballot(want_r && cat_r);
  const unsigned long long mf0 = __ballot(want_f && !cat_f), mf1 = __ballot(want_f && cat_f);
  const unsigned long long below = (1ull << lane) - 1ull;
  unsigned incl = n_s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned t = (unsigned)__shfl_up((int)incl, off, 64);
    if ((int)lane >= off) incl += t;
  }
  const unsigned s_tot = (unsigned)__shfl((int)incl, 63, 64);
  unsigned sb = 0, b0 = 0, b1 = 0, b2 = 0, b3 = 0;
  if (lane == 0) {
    if (s_tot) sb = atomicAdd(a.sh_cnt + s * kShardStride, s_tot);
    if (mr0) b0 = atomicAdd(a.out_cnt + p_r * kShardStride, (unsigned)__popcll(mr0));
    if (mr1) b1 = atomicAdd(a.out_cnt + p_r * kShardStride + 1, (unsigned)__popcll(mr1));
    if (mf0) b2 = atomicAdd(a.out_cnt + p_f * kShardStride, (unsigned)__popcll(mf0));
    if (mf1) b3 = atomicAdd(a.out_cnt + p_f * kShardStride + 1, (unsigned)__popcll(mf1));
  }
  sb = (unsigned)__shfl((int)sb, 0, 64) + (incl - n_s);
  b0 = (unsigned)__shfl((int)b0, 0, 64); b1 = (unsigned)__shfl((int)b1, 0, 64);
  b2 = (unsigned)__shfl((int)b2, 0, 64); b3 = (unsigned)__shfl((int)b3, 0, 64);
  const unsigned r_off = cat_r ? b1 + (unsigned)__popcll(mr1 & below) : b0 + (unsigned)__popcll(mr0 & below);
  const unsigned f_off = cat_f ? b3 + (unsigned)__popcll(mf1 & below) : b2 + (unsigned)__popcll(mf0 & below);
  const unsigned cap = a.out_cap;
  so = sb + n_s <= a.sh_cap ? s * a.sh_cap + sb : ~0u;
  ro = r_off < cap ? p_r * cap + (cat_r ? cap - 1u - r_off : r_off) : ~0u;
  fo = f_off < cap ? p_f * cap + (cat_f ? cap - 1u - f_off : f_off) : ~0u;
}

// Block-wide: the exclusive prefix of a queue's region counts into LDS, or
// nullptr for a dense generation. Every thread of the block calls it (it
// synchronises when cnt != nullptr).
// DUAL = false: the parent (shadow) list, kShards regions, pre[0..kShards].
// DUAL = true: a generation's rays, 2 kShards virtual regions v (shard_append:
// kind half h = v / kShards, end e = (v / (kShards/2)) % 2, region r =
// v % (kShards/2) of the half), pre[0..2 kShards]: each class's regions are
// contiguous in the dense order.
template <bool DUAL>
__device__ __forceinline__ const unsigned* shard_prefix(const unsigned* cnt, unsigned* pre) {
  if (!cnt) return nullptr;
  if (threadIdx.x < 64) {
    const unsigned l = threadIdx.x;
    unsigned va = 0, vb = 0;
    if (DUAL) {
      auto count = [&](unsigned v) {
        const unsigned h = v / kShards, e = (v / (kShards / 2)) & 1u, r = v % (kShards / 2);
        return cnt[(h * (kShards / 2) + r) * kShardStride + e];
      };
      va = count(2 * l);
      vb = count(2 * l + 1);
    } else {
      va = l < kShards ? cnt[l * kShardStride] : 0u;
    }
    unsigned incl = va + vb;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned t = (unsigned)__shfl_up((int)incl, off, 64);
      if ((int)l >= off) incl += t;
    }
    if (DUAL) {
      pre[2 * l + 1] = incl - vb;
      pre[2 * l + 2] = incl;
    } else if (l < kShards) {
      pre[l + 1] = incl;
    }
    if (l == 0) pre[0] = 0;
  }
  __syncthreads();
  return pre;
}
// Slot of the j-th entry of a sharded queue (regions of `cap`), j < the total.
template <bool DUAL>
__device__ __forceinline__ unsigned shard_slot(const unsigned* pre, unsigned cap, unsigned j) {
  if (!pre) return j;
  unsigned lo = 0;
#pragma unroll
  for (unsigned step = DUAL ? kShards : kShards / 2; step > 0; step >>= 1)
    if (pre[lo + step] <= j) lo += step;
  const unsigned off = j - pre[lo];
  if (!DUAL) return lo * cap + off;
  const unsigned h = lo / kShards, e = (lo / (kShards / 2)) & 1u, r = lo % (kShards / 2);
  return (h * (kShards / 2) + r) * cap + (e ? cap - 1u - off : off);
}
constexpr unsigned kPreRays = 2 * kShards + 1, kPreList = kShards + 1;  // LDS prefix sizes

// The frame of generation-0 slot i of a batch (FrameTable) and the slot
// within that frame.
__device__ __forceinline__ unsigned frame_of(const WfArgs& a, unsigned i, unsigned& li) {
  if (a.n_frames <= 1) {
    li = i;
    return 0u;
  }
  const unsigned f = i / a.frame_rays;
  li = i - f * a.frame_rays;
  return f;
}

// Root rays of generation 0: sample `smp` of a pixel of the shard
// (camera.rs:57-69 / 71-90) of the slot's frame, or an explicit ray; deeper
// generations read their queue.
// CAM = false: a launch that never reads camera rays (generations >= 1, or
// explicit rays), compiled without the camera path and its registers.
// NT: the ray's last read (non-temporal: it leaves the L2 to the scene).
template <bool CAM = true, bool NT = true>
__device__ __forceinline__ void wf_ray(const WfArgs& a, const DevCamera& cam, unsigned i, V3& o, V3& d) {
  if (CAM && a.g == 0 && a.camera_mode) {
    unsigned li;
    const unsigned f = frame_of(a, i, li);
    const DevCamera& cf = a.n_frames > 1 ? a.frames->cam[f] : cam;
    uint32_t x, lr, smp;
    gen0_pixel(a.aa, a.rows, cf.hsize, li, x, lr, smp);
    const uint32_t blk = lr / a.row_block, off = lr - blk * a.row_block;
    uint32_t gb = blk * a.n_shards + a.shard;  // the canvas block of local block blk
    if (a.blk_period) {  // a block pattern: the j-th set bit of the mask in period k
      unsigned long long m = a.blk_mask;
      const uint32_t per = (uint32_t)__popcll(m), k = blk / per;
      uint32_t j = blk - k * per, pos = 0;
#pragma unroll
      for (uint32_t w = 32; w >= 1; w >>= 1) {
        const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
        if (j >= c) { j -= c; m >>= w; pos += w; }
      }
      gb = k * a.blk_period + pos;
    }
    const uint32_t y = gb * a.row_block + off;
    if (a.aa == 1) {
      ray_for_pixel(cf, x, y, o, d);
    } else {
      const double* ofs = kAaOffsets[a.aa - 1 + smp];
      ray_for_pixel(cf, x, y, o, d, ofs[0], ofs[1]);
    }
  } else {
    const f64x2* r = reinterpret_cast<const f64x2*>(a.rays + i);  // 48 B, 16-B aligned
    f64x2 r0, r1, r2;
    if constexpr (NT) {
      r0 = __builtin_nontemporal_load(r); r1 = __builtin_nontemporal_load(r + 1); r2 = __builtin_nontemporal_load(r + 2);
    } else {
      r0 = r[0]; r1 = r[1]; r2 = r[2];
    }
    o = v3(r0.x, r0.y, r1.x);
    d = v3(r1.y, r2.x, r2.y);
  }
}

// Shadow ray j of a generation: World::is_shadowed(comps.over_point, light)
// (world.rs:95-105) for shadow slot a.shadow_nodes[j] = node * L + light,
// built from the node's over point exactly as the reference builds it
// (v = light - point, distance = |v|, direction = v.normalize()).
__device__ __forceinline__ void shadow_ray(const DevScene& sc, const WfArgs& a, unsigned j, V3& o, V3& d,
                                           double& dist, unsigned& slot, unsigned* light = nullptr) {
  const unsigned L = (unsigned)sc.n_lights;
  slot = (unsigned)a.shadow_nodes[j];
  const unsigned node = L == 1 ? slot : slot / L, l = slot - node * L;
  if (light) *light = l;
  const double* ov = a.geo[node].over;
  o = v3(ov[0], ov[1], ov[2]);
  cLightRec Lr = (cLightRec)sc.lights + l;
  const V3 v = vsub(v3(Lr->pos[0], Lr->pos[1], Lr->pos[2]), o);
  dist = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);  // magnitude (vector.rs:21-23)
  d = vnormalize(v);
}

// The outcome of shadow ray `slot` (= node slot * L + light): lighting() of
// the hit with that light (material.rs:38-82), in shadow or not, as the
// reference's shade_hit evaluates it (world.rs:41-56).
// `over` and `lightv` are the shadow ray's origin and direction (shadow_ray):
// the over point and the light vector lighting() would recompute.
__device__ __forceinline__ void shadow_result(const DevScene& sc, const WfArgs& a, unsigned slot, bool shadowed,
                                              V3 over, V3 lightv) {
  const unsigned L = (unsigned)sc.n_lights;
  const unsigned node = L == 1 ? slot : slot / L, l = slot - node * L;
  const WfGeo& g = a.geo[node];
  const V3 c = lighting(sc.shade[g.obj], (cLightRec)sc.lights + l, over, v3(g.eyev[0], g.eyev[1], g.eyev[2]),
                        v3(g.normal[0], g.normal[1], g.normal[2]), shadowed, lightv);
  double* dst = a.surf + (size_t)slot * 3;
  dst[0] = c.x; dst[1] = c.y; dst[2] = c.z;
}


// ------------------------------------------------------------ primary records
// Per diagonal sphere: s (inverse diagonal), o' = s*o + t for the camera origin
// o, and c = o'.o' - 1 — the same operations the general test performs, so the
// values are bit-identical to what each primary ray would compute.
// The frame's first launch: zero the work counters and the queue counters of
// this workspace (n_a and n_b 16-B words) and, for a camera frame, write the
// primary records (wf_prim_prep's computation). One launch instead of two
// fills and a kernel.
#ifndef RT_WF_GLOBAL_TU
// A batch of frames (n_frames > 1) also writes the batch's FrameTable, passed
// by value (so the host may reuse its copy at once), to the workspace's
// device copy that the pass's later launches read, and one set of primary
// records per frame (frame f's at prim + f * (n_diag + 4)).
// A fast-path frame also places generation 0 (WfGenTab, device-sized
// generations): dense, its colours and parents at the arenas' start.
__global__ void wf_frame_init(DevScene sc, DevCamera cam, PrimRec* prim, unsigned do_prim, uint4* zero_a,
                              unsigned n_a, uint4* zero_b, unsigned n_b, FrameTable tab, FrameTable* tab_dev,
                              unsigned n_frames, WfGenTab* gtab) {
  const unsigned stride = gridDim.x * blockDim.x;
  const unsigned i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
  if (gtab && i0 == 0) gtab[0] = WfGenTab{0u, 0u, 0ull, 0ull};
  for (unsigned i = i0; i < n_a; i += stride) zero_a[i] = z;
  for (unsigned i = i0; i < n_b; i += stride) zero_b[i] = z;
  if (n_frames > 1) {
    const unsigned* src = (const unsigned*)&tab;
    unsigned* dst = (unsigned*)tab_dev;
    for (unsigned i = i0; i < (unsigned)(sizeof(FrameTable) / 4); i += stride) dst[i] = src[i];
  }
  if (!do_prim) return;
  const unsigned per = (unsigned)sc.n_diag + 4;
  for (unsigned jj = i0; jj < per * n_frames; jj += stride) {
    const unsigned f = jj / per, j = jj - f * per;
    const V3 o = m34_point(n_frames > 1 ? tab.cam[f].inv : cam.inv, v3(0.0, 0.0, 0.0));  // camera.rs:65
    PrimRec p{};
    if (j < (unsigned)sc.n_diag) {
      const SphereDiag& r = sc.sph_diag[j];
      p.s[0] = r.s[0]; p.s[1] = r.s[1]; p.s[2] = r.s[2];
      p.op[0] = r.s[0] * o.x + r.t[0];
      p.op[1] = r.s[1] * o.y + r.t[1];
      p.op[2] = r.s[2] * o.z + r.t[2];
      p.c = p.op[0] * p.op[0] + p.op[1] * p.op[1] + p.op[2] * p.op[2] - 1.0;
    }
    prim[jj] = p;  // j >= n_diag: zero padding records
  }
}
#endif

// LDS image for the trace kernels: [diag or prim records][gen][planes][metas]
struct WfLds {
  const double* diag;  // 6 doubles per record (general) or 8 (primary)
  const double* gen;
  const double* plane;
  const int* diag_meta;
  const int* gen_meta;
  const int* plane_meta;
};
__host__ __device__ inline size_t wf_lds_bytes(int nd, int ng, int np, bool primary) {
  return lds_align16((size_t)(nd + 4) * (primary ? 64 : 48)) + lds_align16((size_t)ng * 96) +
         lds_align16((size_t)np * 32) + lds_align16((size_t)nd * 4) + lds_align16((size_t)ng * 4) +
         lds_align16((size_t)np * 4);
}
template <bool PRIMARY>
__device__ WfLds wf_lds_stage(const DevScene& sc, const PrimRec* prim, unsigned char* base) {
  WfLds v;
  size_t off = 0;
  const int rec = PRIMARY ? 8 : 6;
  v.diag = (const double*)(base + off); off += lds_align16((size_t)(sc.n_diag + 4) * rec * 8);
  v.gen = (const double*)(base + off); off += lds_align16((size_t)sc.n_gen * 96);
  v.plane = (const double*)(base + off); off += lds_align16((size_t)sc.n_planes * 32);
  v.diag_meta = (const int*)(base + off); off += lds_align16((size_t)sc.n_diag * 4);
  v.gen_meta = (const int*)(base + off); off += lds_align16((size_t)sc.n_gen * 4);
  v.plane_meta = (const int*)(base + off);
  double* dd = (double*)v.diag;
  if constexpr (PRIMARY) {
    const double* src = (const double*)prim;
    for (int i = threadIdx.x; i < (sc.n_diag + 4) * 8; i += blockDim.x) dd[i] = src[i];
  } else {
    for (int i = threadIdx.x; i < (sc.n_diag + 4) * 6; i += blockDim.x) {
      const int r = i / 6, e = i - r * 6;
      dd[i] = r >= sc.n_diag ? 0.0 : e < 3 ? sc.sph_diag[r].s[e] : sc.sph_diag[r].t[e - 3];
    }
  }
  for (int i = threadIdx.x; i < sc.n_gen * 12; i += blockDim.x) ((double*)v.gen)[i] = sc.sph_gen[i / 12].m[i % 12];
  for (int i = threadIdx.x; i < sc.n_planes * 4; i += blockDim.x) ((double*)v.plane)[i] = sc.planes[i / 4].m[i % 4];
  for (int i = threadIdx.x; i < sc.n_diag; i += blockDim.x) ((int*)v.diag_meta)[i] = (int)sc.sph_diag[i].meta;
  for (int i = threadIdx.x; i < sc.n_gen; i += blockDim.x) ((int*)v.gen_meta)[i] = (int)sc.sph_gen[i].meta;
  for (int i = threadIdx.x; i < sc.n_planes; i += blockDim.x) ((int*)v.plane_meta)[i] = (int)sc.planes[i].meta;
  __syncthreads();
  return v;
}

// World::intersect + hit over the LDS image (closest hit + containers top-2,
// or the shadow-caster variant). Sphere records are read as wave-uniform
// ds_read_b128 broadcasts with a one-record look-ahead; the image holds zero
// padding records, so record j+1 always exists.
template <bool PRIMARY, bool SHADOW, bool QUADS>
__device__ __forceinline__ void wf_trace_lds(const DevScene& sc, const WfLds& lv, V3 o, V3 d, Hit& h,
                                             unsigned& n_disc, GateSkips& sk) {
  hit_init(h);
  const d2* r = (const d2*)lv.diag;
  if constexpr (PRIMARY) {
    // record: (s0 s1) (s2 o'x) (o'y o'z) (c pad); 16 f64 ops per test
    d2 a0 = r[0], a1 = r[1], a2 = r[2], a3 = r[3];
    int j = 0;
    for (; j + 1 < sc.n_diag; j += 2) {
      const d2 b0 = r[4 * j + 4], b1 = r[4 * j + 5], b2 = r[4 * j + 6], b3 = r[4 * j + 7];
      {
        const double dx = a0.x * d.x, dy = a0.y * d.y, dz = a1.x * d.z;
        sphere_adc<SHADOW>(dx * dx + dy * dy + dz * dz, dx * a1.y + dy * a2.x + dz * a2.y, a3.x,
                           [&] { return lv.diag_meta[j]; }, h, n_disc);
      }
      a0 = r[4 * j + 8]; a1 = r[4 * j + 9]; a2 = r[4 * j + 10]; a3 = r[4 * j + 11];
      {
        const double dx = b0.x * d.x, dy = b0.y * d.y, dz = b1.x * d.z;
        sphere_adc<SHADOW>(dx * dx + dy * dy + dz * dz, dx * b1.y + dy * b2.x + dz * b2.y, b3.x,
                           [&] { return lv.diag_meta[j + 1]; }, h, n_disc);
      }
    }
    if (j < sc.n_diag) {
      const double dx = a0.x * d.x, dy = a0.y * d.y, dz = a1.x * d.z;
      sphere_adc<SHADOW>(dx * dx + dy * dy + dz * dz, dx * a1.y + dy * a2.x + dz * a2.y, a3.x,
                         [&] { return lv.diag_meta[j]; }, h, n_disc);
    }
  } else {
    // record: (s0 s1) (s2 t0) (t1 t2); 28 f64 ops per test
    d2 a0 = r[0], a1 = r[1], a2 = r[2];
    int j = 0;
    for (; j + 1 < sc.n_diag; j += 2) {
      const d2 b0 = r[3 * j + 3], b1 = r[3 * j + 4], b2 = r[3 * j + 5];
      sphere_test<SHADOW>(a0.x * o.x + a1.y, a0.y * o.y + a2.x, a1.x * o.z + a2.y, a0.x * d.x, a0.y * d.y,
                          a1.x * d.z, [&] { return lv.diag_meta[j]; }, h, n_disc);
      a0 = r[3 * j + 6]; a1 = r[3 * j + 7]; a2 = r[3 * j + 8];
      sphere_test<SHADOW>(b0.x * o.x + b1.y, b0.y * o.y + b2.x, b1.x * o.z + b2.y, b0.x * d.x, b0.y * d.y,
                          b1.x * d.z, [&] { return lv.diag_meta[j + 1]; }, h, n_disc);
    }
    if (j < sc.n_diag)
      sphere_test<SHADOW>(a0.x * o.x + a1.y, a0.y * o.y + a2.x, a1.x * o.z + a2.y, a0.x * d.x, a0.y * d.y,
                          a1.x * d.z, [&] { return lv.diag_meta[j]; }, h, n_disc);
  }
  for (int j = 0; j < sc.n_gen; ++j) {
    const int gate = ((cSphereGen)sc.sph_gen)[j].gate;  // (shapes inside groups: group_gate)
    if (gate && !group_gate(sc, gate, o, d)) { ++sk.sph; continue; }
    double m[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) m[e] = lv.gen[12 * j + e];
    const V3 lo = m34_point(m, o);
    const V3 ld = v3(m[0] * d.x + m[1] * d.y + m[2] * d.z, m[4] * d.x + m[5] * d.y + m[6] * d.z,
                     m[8] * d.x + m[9] * d.y + m[10] * d.z);
    sphere_test<SHADOW>(lo.x, lo.y, lo.z, ld.x, ld.y, ld.z, [&] { return lv.gen_meta[j]; }, h, n_disc);
  }
  for (int j = 0; j < sc.n_planes; ++j) {  // plane.rs:53-60
    const int gate = ((cPlaneRec)sc.planes)[j].gate;
    if (gate && !group_gate(sc, gate, o, d)) { ++sk.plane; continue; }
    const double m0 = lv.plane[4 * j], m1 = lv.plane[4 * j + 1], m2 = lv.plane[4 * j + 2], m3 = lv.plane[4 * j + 3];
    plane_test<SHADOW>(m0 * o.x + m1 * o.y + m2 * o.z + m3, m0 * d.x + m1 * d.y + m2 * d.z, lv.plane_meta[j], h);
  }
  if constexpr (QUADS) {
    cQuadRec qr = (cQuadRec)sc.quads;  // cubes / cylinders / cones: scalar loads
    for (int j = 0; j < sc.n_quads; ++j) {
      if (qr[j].gate && !group_gate(sc, qr[j].gate, o, d)) { ++sk.other; continue; }
      quad_test<SHADOW>(qr + j, o, d, h);
    }
  }
  hit_finish(h);
}

// The counted launches' group skips (GateSkips), summed per wave into the
// calling wave's counter row.
__device__ __forceinline__ void add_gate_skips(WfCounters* cnt, const GateSkips& sk) {
  const unsigned long long a = wave_sum(sk.sph), b = wave_sum(sk.plane), c = wave_sum(sk.other);
  if (lane_id() == 0 && (a | b | c)) {
    WfWorkRow* w = work_row(cnt);
    if (a) atomicAdd(&w->gated[0], a);
    if (b) atomicAdd(&w->gated[1], b);
    if (c) atomicAdd(&w->gated[2], c);
  }
}

// ---------------------------------------------------------- trace kernels
template <bool USE_LDS, bool PRIMARY, bool QUADS, int TW>
__global__ __launch_bounds__(kTraceBlock, TW) void wf_trace_closest(DevScene sc, DevCamera cam, WfArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  unsigned n_disc = 0;
  GateSkips sk;
  WfLds lv{};
  if constexpr (USE_LDS) lv = wf_lds_stage<PRIMARY>(sc, a.prim, lds_raw);
  __shared__ unsigned s_pre[kPreRays];
  const unsigned* pre = shard_prefix<true>(a.in_cnt, s_pre);
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const unsigned slot = shard_slot<true>(pre, a.in_cap, i);
    V3 o, d;
    wf_ray(a, cam, slot, o, d);
    Hit h;
    if constexpr (USE_LDS) wf_trace_lds<PRIMARY, false, QUADS>(sc, lv, o, d, h, n_disc, sk);
    else trace<false>(sc, o, d, h, n_disc, &sk);
    WfHit w;
    w.t = h.t; w.key = h.key; w.c1k = h.c1k; w.c2k = h.c2k; w.hin = h.hin;
    a.hits[slot] = w;
  }
  const unsigned long long s = wave_sum(n_disc);
  if (lane_id() == 0 && s) atomicAdd(&work_row(a.cnt)->disc[a.disc_slot], s);
  if (sc.n_groups) add_gate_skips(a.cnt, sk);
}

// World::is_shadowed (world.rs:95-105): shadowed iff some shadow-casting
// object has a root t with 0 <= t < distance (the first t >= 0 among shadow
// casters in the sorted list is the minimum one). Full traversal: the exact
// counters (sphere_disc_ge0) need every test.
template <bool USE_LDS, bool QUADS, int TW>
__global__ __launch_bounds__(kTraceBlock, TW) void wf_trace_shadow(DevScene sc, WfArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  unsigned n_disc = 0;
  GateSkips sk;
  WfLds lv{};
  if constexpr (USE_LDS) lv = wf_lds_stage<false>(sc, nullptr, lds_raw);
  __shared__ unsigned s_pre[kPreList];
  const unsigned* pre = shard_prefix<false>(a.sh_cnt, s_pre);
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n_shadow; i += stride) {
    V3 o, d;
    double dist;
    unsigned slot;
    shadow_ray(sc, a, shard_slot<false>(pre, a.sh_cap, i), o, d, dist, slot);
    Hit h;
    if constexpr (USE_LDS) wf_trace_lds<false, true, QUADS>(sc, lv, o, d, h, n_disc, sk);
    else trace<true>(sc, o, d, h, n_disc, &sk);
    shadow_result(sc, a, slot, h.key >= 0 && h.t < dist, o, d);
  }
  const unsigned long long s = wave_sum(n_disc);
  if (lane_id() == 0 && s) atomicAdd(&work_row(a.cnt)->disc[a.disc_slot], s);
  if (sc.n_groups) add_gate_skips(a.cnt, sk);
}

// The classes of a node's children in the next generation's queue (shard_append):
// a reflection off a plane (a mirror image of the incoming rays: coherent) or
// off anything else; a refraction leaving an object (the hit was from inside)
// or entering one.
__device__ __forceinline__ bool ray_class_r(const DevScene& sc, bool hit, const Comps& c) {
  return hit && sc.shade[c.obj].kind == 1;  // RT_SHAPE_PLANE
}
__device__ __forceinline__ bool ray_class_f(bool hit, const Comps& c) { return hit && c.inside; }

// ---------------------------------------------------------- prep (spawn)
// prepare_computations (intersection.rs:53-105) of ray i's finished hit `h`
// (stored at `slot`) and the spawn of its shadow, reflected and refracted rays
// (world.rs:40-134): the hit node, the shadow-list entries and the next
// generation's rays. Every lane of the wave calls it (shard_append), `valid`
// false for the padding lanes. wf_prep runs it on the stored hits; the BVH
// trace kernels run it right after their traversal (no hit queue).
__device__ __forceinline__ void prep_one(const DevScene& sc, const WfArgs& a, unsigned i, unsigned slot, bool valid,
                                         V3 o, V3 d, const Hit& h) {
  const unsigned L = (unsigned)sc.n_lights;
  const unsigned remaining = a.max_depth - a.g;
  bool hit = false, want_refl = false, want_refr = false;
  Comps c{};
  V3 refr_dir = v3(0, 0, 0);
  const ShadeRec* m = nullptr;
  if (valid) {
    if (h.key >= 0) {
      c = prepare(sc, o, d, h);
      hit = true;
      m = &sc.shade[c.obj];
      // reflected_color (world.rs:107-114)
      want_refl = !(req(m->reflective, 0.0) || remaining == 0);
      // refracted_color (world.rs:116-134)
      if (!(req(m->transparency, 0.0) || remaining == 0)) {
        const double n_ratio = c.n1 / c.n2;
        const double cos_i = vdot(c.eyev, c.normal);
        const double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
        if (!(sin2_t > 1.0)) {
          const double cos_t = sqrt(1.0 - sin2_t);
          refr_dir = vsub(vscale(c.normal, n_ratio * cos_i - cos_t), vscale(c.eyev, n_ratio));
          want_refr = true;
        }
      }
    }
  }
  // shadow rays: one per light (world.rs:41-56); the fast path leaves out the
  // ones whose answer cannot change the colour, and their lighting() value
  // (the ambient term) is written here; the shadow trace writes the others
  unsigned n_s = 0, skip = 0;
  if (hit) {
    for (unsigned l = 0; l < L; ++l) {
      V3 amb;
      cLightRec Lr = (cLightRec)sc.lights + l;
      if (a.skip_shadow && l < 32 &&
          shadow_irrelevant(*m, Lr, vnormalize(vsub(v3(Lr->pos[0], Lr->pos[1], Lr->pos[2]), c.over)), c.normal, amb)) {
        skip |= 1u << l;
        double* sp = a.surf + ((size_t)slot * L + l) * 3;
        sp[0] = amb.x; sp[1] = amb.y; sp[2] = amb.z;
      } else {
        ++n_s;
      }
    }
  }
  unsigned sbase, rbase, fbase;
  shard_append(a, i / 64, n_s, want_refl, want_refr, sbase, rbase, fbase, ray_class_r(sc, hit, c),
               ray_class_f(hit, c));
  if (!valid) return;
  WfNode nd;
  nd.obj = -1; nd.child_refl = -1; nd.child_refr = -1; nd.pad = 0; nd.schlick = 0.0;
  if (hit) {
    nd.obj = c.obj;
    if (n_s) {
      WfGeo gm;
      gm.over[0] = c.over.x; gm.over[1] = c.over.y; gm.over[2] = c.over.z;
      gm.normal[0] = c.normal.x; gm.normal[1] = c.normal.y; gm.normal[2] = c.normal.z;
      gm.eyev[0] = c.eyev.x; gm.eyev[1] = c.eyev.y; gm.eyev[2] = c.eyev.z;
      gm.obj = c.obj; gm.pad = 0;
      a.geo[slot] = gm;
    }
    // shade_hit's Schlick factor (world.rs:62-64), same inputs as the reference's call
    nd.schlick = (m->reflective > 0.0 && m->transparency > 0.0) ? schlick(c.eyev, c.normal, c.n1, c.n2) : 0.0;
    for (unsigned l = 0; l < L; ++l)  // its shadow rays are built by the shadow trace
      if (!(l < 32 && (skip >> l & 1u)) && sbase != ~0u) a.shadow_nodes[sbase++] = (int32_t)(slot * L + l);
    if (want_refl && rbase != ~0u) {
      const V3 rv = vreflect(d, c.normal);  // comps.reflectv (intersection.rs:101)
      WfRay r;
      r.o[0] = c.over.x; r.o[1] = c.over.y; r.o[2] = c.over.z;
      r.d[0] = rv.x; r.d[1] = rv.y; r.d[2] = rv.z;
      a.next_rays[rbase] = r;
      nd.child_refl = (int)rbase;
    }
    if (want_refr && fbase != ~0u) {
      WfRay r;
      r.o[0] = c.under.x; r.o[1] = c.under.y; r.o[2] = c.under.z;
      r.d[0] = refr_dir.x; r.d[1] = refr_dir.y; r.d[2] = refr_dir.z;
      a.next_rays[fbase] = r;
      nd.child_refr = (int)fbase;
    }
  }
  a.nodes[slot] = nd;
}

// ------------------------------------------------------------ fused trace kernels
// The fast path (BVH) evaluates a whole generation in ONE launch per
// generation (DESIGN.md "Fused generations"): closest hit, prepare_computations,
// the child-ray spawn, every light's shadow ray and lighting(), and, for a
// node without children (a miss, a diffuse surface, the last generation), its
// final colour. Only nodes with a reflected or refracted child are queued
// (ParentRec) for wf_combine_parents, which runs once the children's colours
// exist. Scene images of the kernels (LANE):
//   15: the four-wide hierarchy + 48-B sphere records + 16-bit stack in LDS
//       (the default where they fit)
//   14: pair-layout nodes + sphere records + per-lane stack in LDS
//    4: the four-wide hierarchy and records in global memory, a treelet of its
//       top nodes and the 16-bit stack in LDS (the default for larger scenes)
//    3: binary nodes and records in global memory, per-lane stack in LDS
//    1: nodes and records in global memory, per-lane stack in scratch (trees
//       deeper than kLaneLdsDepth)
//    0: primary rays, wave (packet) traversal over global nodes (one LDS stack
//       per wave); the sphere records are staged in LDS for the shadow rays
//       when they fit
// The per-light box distances of the light buffer are staged in LDS when they
// fit beside the image (WfArgs::lds_flags).
// Where generation g's colour of ray `slot` goes: generation 0 of a camera
// render without AA is tile-ordered, and its colours are written row-major
// into the output.
template <bool CAM = true>
__device__ __forceinline__ double* color_dst(const WfArgs& a, const DevCamera& cam, unsigned slot) {
  size_t oi = slot;
  if (CAM && a.g == 0 && a.camera_mode && a.aa == 1) {
    unsigned li;
    const unsigned f = frame_of(a, slot, li);
    uint32_t x, lr, smp;
    gen0_pixel(1u, a.rows, cam.hsize, li, x, lr, smp);
    oi = (size_t)lr * cam.hsize + x;
    if (a.n_frames > 1) return a.frames->out[f] + oi * 3;
  }
  return a.colors + oi * 3;
}

__device__ __forceinline__ void st_ray(WfRay* p, V3 o, V3 d) {
  f64x2* q = reinterpret_cast<f64x2*>(p);  // 48 B, 16-B aligned
  __builtin_nontemporal_store((f64x2){o.x, o.y}, q);
  __builtin_nontemporal_store((f64x2){o.z, d.x}, q + 1);
  __builtin_nontemporal_store((f64x2){d.y, d.z}, q + 2);
}

// Device-sized generations (DESIGN.md "Device-sized generations"): the
// launch of generation g takes its ray count from the queue counters (`pre`,
// the prefix of its regions; generation 0: the host's count), sizes the
// regions of generation g+1 and of its own parent list from it exactly as
// the capacity argument of shard_append needs ("Sharded queues": a region of
// the next generation takes at most 2 `per` wave-iterations of at most 64 rays
// of its kind, a parent region at most `per` of at most 64 parents), and
// places them after generation g's colours and parents in the arenas. Every
// block computes the same values from the same counters and table entry;
// block 0 writes them for the later launches (generation g+1 and the
// combines). A generation whose children or parents do not fit spawns none
// (out_cap = sh_cap = 0: shard_append then hands out no slot, so nothing is
// written out of bounds) and raises the workspace's overflow record; the
// frame is incomplete and the host re-renders it (synchronous calls) or
// reports it (rt_scene_check). Returns the generation's ray count.
__device__ __forceinline__ unsigned bind_generation(WfArgs& a, const unsigned* pre) {
  const unsigned g = a.g;
  const WfGenTab t = a.gtab[g];
  // (the region counters count every child asked for, also those a full
  // region refused: a generation placed with no room (cap 0, after an
  // overflow) has no rays)
  const unsigned n = g == 0 ? a.n
                            : (pre && t.cap ? (unsigned)__builtin_amdgcn_readfirstlane((int)pre[2 * kShards]) : 0u);
  const unsigned groups = ((n + 63u) / 64u + kShardGroup - 1u) / kShardGroup;
  const unsigned per = kShardGroup * ((groups + kShards - 1u) / kShards);
  // the last generation spawns no children, so it has no parents either
  unsigned out_cap = g < a.max_depth ? 128u * per : 0u, sh_cap = g < a.max_depth ? 64u * per : 0u;
  const unsigned long long slots = g == 0 ? (unsigned long long)n : (unsigned long long)kShards * t.cap;
  const unsigned long long c_next = t.color_off + slots;
  const unsigned long long need_c = c_next + (unsigned long long)kShards * out_cap;
  const unsigned long long need_p = t.par_off + (unsigned long long)kShards * sh_cap;
  const unsigned long long need_r = (unsigned long long)kShards * out_cap;
  const bool fits = need_c <= a.color_cap && need_p <= a.par_cap && need_r <= a.ray_cap;
  if (!fits) { out_cap = 0u; sh_cap = 0u; }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.gsh[g] = sh_cap;
    a.gtab[g + 1] = WfGenTab{out_cap, 0u, c_next, t.par_off + (unsigned long long)kShards * sh_cap};
    if (!fits) {  // host-mapped: plain vector stores, the flag last
      a.cnt->overflow = 1u;  // this pass's canvases are poisoned at its end (poison_frames)
      volatile WfHostRec* r = a.hrec;
      r->need_colors = need_c;
      r->need_parents = need_p;
      r->need_rays = need_r;
      __threadfence_system();
      r->overflow = 1;
    }
  }
  a.n = n;
  a.in_cap = t.cap;
  a.out_cap = out_cap;
  a.sh_cap = sh_cap;
  // (constant indices: a dynamic index would keep the whole argument block in scratch)
  WfRay* const rb0 = a.ray_buf[0];
  WfRay* const rb1 = a.ray_buf[1];
  a.rays = (g & 1u) ? rb1 : rb0;
  a.next_rays = (g & 1u) ? rb0 : rb1;
  if (!(g == 0 && a.colors_direct)) a.colors = a.color_base + t.color_off * 3ull;
  a.parents = a.par_base + t.par_off;
  return n;
}

// Per-lane tallies of a fused trace kernel (summed per wave at the end).
struct FusedTally {
  GateSkips gsk;                                     // shapes groups kept out of a ray (counted launches)
  unsigned disc = 0, tests = 0, boxes = 0;           // closest-hit work
  unsigned sh_disc = 0, sh_tests = 0, sh_boxes = 0;  // shadow-ray work
  unsigned sh_rays = 0;                              // shadow rays traced
  unsigned hits = 0, refl = 0, refr = 0;             // counted launches: shade_hit runs, children spawned
};

// Everything after the closest hit of ray `slot` (index i of the generation):
// prepare_computations (intersection.rs:53-105), the reflected / refracted
// children (world.rs:107-134), shade_hit's lighting over the lights in order
// (world.rs:40-56: one is_shadowed per light, a left fold from black), then
// either the final colour (no children) or a ParentRec. Every lane of the wave
// calls it (shard_append), `valid` false for the padding lanes.
template <int LANE, bool QUADS, bool CAM>
__device__ __forceinline__ void shade_fused(const DevScene& sc, const DevCamera& cam, const WfArgs& a,
                                            const LaneScene& ls, unsigned q, unsigned slot, bool valid, V3 o, V3 d,
                                            const Hit& h, FusedTally& t) {
  const unsigned L = (unsigned)sc.n_lights;
  const unsigned remaining = a.max_depth - a.g;
  bool hit = false, want_refl = false, want_refr = false;
  Comps c{};
  V3 refr_dir = v3(0, 0, 0);
  const ShadeRec* m = nullptr;
  if (valid && h.key >= 0) {
    c = prepare(sc, o, d, h);
    hit = true;
    m = &sc.shade[c.obj];
    // reflected_color (world.rs:107-114)
    want_refl = !(req(m->reflective, 0.0) || remaining == 0);
    // refracted_color (world.rs:116-134)
    if (!(req(m->transparency, 0.0) || remaining == 0)) {
      const double n_ratio = c.n1 / c.n2;
      const double cos_i = vdot(c.eyev, c.normal);
      const double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
      if (!(sin2_t > 1.0)) {
        const double cos_t = sqrt(1.0 - sin2_t);
        refr_dir = vsub(vscale(c.normal, n_ratio * cos_i - cos_t), vscale(c.eyev, n_ratio));
        want_refr = true;
      }
    }
  }
  const bool parent = want_refl || want_refr;
  unsigned pbase, rbase, fbase;
  shard_append(a, q, parent ? 1u : 0u, want_refl, want_refr, pbase, rbase, fbase, ray_class_r(sc, hit, c),
               ray_class_f(hit, c));
  if (!valid) return;
  t.hits += hit; t.refl += want_refl; t.refr += want_refr;
  double* dst = color_dst<CAM>(a, cam, slot);
  if (!hit) {  // color_at: a miss is black (world.rs:74-75)
    st_d(dst, 0.0); st_d(dst + 1, 0.0); st_d(dst + 2, 0.0);
    return;
  }
  int child_refl = -1, child_refr = -1;
  if (want_refl && rbase != ~0u) {
    st_ray(a.next_rays + rbase, c.over, vreflect(d, c.normal));  // comps.reflectv (intersection.rs:101)
    child_refl = (int)rbase;
  }
  if (want_refr && fbase != ~0u) {
    st_ray(a.next_rays + fbase, c.under, refr_dir);
    child_refr = (int)fbase;
  }
  // shade_hit's Schlick factor (world.rs:62-64), same inputs as the reference's call
  const double schlick_r =
      (m->reflective > 0.0 && m->transparency > 0.0) ? schlick(c.eyev, c.normal, c.n1, c.n2) : 0.0;
  // surface = Sum over the lights of lighting(..., is_shadowed(over_point, light))
  V3 surface = v3(0.0, 0.0, 0.0);  // fold from (0,0,0) (color.rs:96-103)
  for (unsigned l = 0; l < L; ++l) {
    cLightRec Lr = (cLightRec)sc.lights + l;
    // the shadow ray exactly as World::is_shadowed builds it (world.rs:95-105); its
    // direction is also lighting()'s light vector (same operands, same operations)
    const V3 v = vsub(v3(Lr->pos[0], Lr->pos[1], Lr->pos[2]), c.over);
    const double dist = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);  // magnitude (vector.rs:21-23)
    const V3 sdir = v3(v.x / dist, v.y / dist, v.z / dist);       // normalize (vector.rs:25-28)
    V3 term;
    if (a.skip_shadow && shadow_irrelevant(*m, Lr, sdir, c.normal, term)) {
      // the light is behind the surface: lighting() is the ambient term either way
    } else {
      const bool shadowed = shadow_trace<LANE, QUADS>(sc, a.use_lb, ls, l, c.over, sdir, dist, t.sh_disc, t.sh_tests,
                                                      t.sh_boxes, &t.gsk);
      if (QUADS && a.count) count_hier_gates(sc, c.over, sdir, t.gsk);
      ++t.sh_rays;
      term = lighting(*m, Lr, c.over, c.eyev, c.normal, shadowed, sdir);
    }
    surface = vadd(surface, term);
  }
  if (child_refl >= 0 || child_refr >= 0) {  // the children's colours come later (wf_combine_parents)
    if (pbase != ~0u) {
      ParentRec* pr = a.parents + pbase;
      st_d(&pr->surface[0], surface.x); st_d(&pr->surface[1], surface.y); st_d(&pr->surface[2], surface.z);
      st_d(&pr->schlick, schlick_r);
      i32x4 tail = {(int)slot, c.obj, child_refl, child_refr};
      __builtin_nontemporal_store(tail, (i32x4*)&pr->slot);
    }
    return;
  }
  const V3 zero = v3(0.0, 0.0, 0.0);  // reflected / refracted colour: black (world.rs:108-109, 117-118)
  const V3 col = shade_color(*m, surface, zero, zero, schlick_r);
  st_d(dst, col.x); st_d(dst + 1, col.y); st_d(dst + 2, col.z);
}

// One generation of the fast path (see above). PRIMARY: generation 0 of a
// camera render (wave traversal with the shared-origin primary records).
// TALLY: the launch sums its executed work (counted launches: stats asked
// for). Every other frame (the timed ones, the profiled ones) skips the
// per-visit and per-test counting and the wave-end atomics altogether: C3
// 1.021 -> 0.964 ms/frame, an 8-way shard 0.204 -> 0.184 ms.
// CAM: the launch may read camera rays (generation 0 of a camera render).
template <bool PRIMARY, bool QUADS, int LANE, bool TALLY, bool CAM = PRIMARY>
__global__ __launch_bounds__(kTraceBlock, 4) void wf_trace_fused(DevScene sc, DevCamera cam, WfArgs a) {
  __shared__ int stack_lds[LANE == 3 ? kLaneLdsDepth * kTraceBlock
                           : LANE == 0 ? (kTraceBlock / 64) * (kBvhMaxDepth + 4) : 1];
  extern __shared__ __attribute__((aligned(16))) unsigned char lane_dyn[];
  int* stk = LANE == 0 ? stack_lds + (threadIdx.x / 64) * (kBvhMaxDepth + 4) : stack_lds + threadIdx.x;
  __shared__ unsigned s_pre[kPreRays];
  const unsigned* pre = shard_prefix<true>(a.in_cnt, s_pre);
  if (a.dev_sized) bind_generation(a, pre);
  // a block without a chunk (static split below: its first chunk lies past the
  // last) leaves before staging the image; the exit is block-uniform
  if (blockIdx.x * (blockDim.x / 64u) >= (a.n + 63u) / 64u) return;
  const LaneScene ls = lane_scene<LANE>(sc, a.lds_flags, a.n_top, stk, lane_dyn);
  FusedTally t;
  // Work distribution: chunk c = rays [64c, 64c + 64), one wave-iteration.
  // A launch with more chunks than waves hands them out dynamically from the
  // counter of the wave's block class (blocks are dealt round-robin to the 8
  // XCDs): class x holds the chunks x + X k. A wave that finishes early takes
  // the next chunk, so the launch ends with the last chunk, not with the
  // slowest wave of a static split (an LDS image holds its CU until every wave
  // of its block is done): C3 1.098 -> 1.013 ms/frame. The next chunk is asked
  // for when the current one starts. A launch with one to three chunks per
  // wave (the deep generations; most generations of a 2-way shard) gives each
  // wave its first chunk statically (chunk = wave index, no atomic to wait
  // for) and hands out the rest, W + x + X k, from the class counters: a
  // 2-way shard 0.554 -> 0.540 ms/frame; the same form for the large launches
  // cost 1.5 % on C3 (their chunks then leave the class-interleaved order).
  // A launch with at most one chunk per wave (an 8-way shard's deep
  // generations) strides over them statically, with no atomics.
  // Every lane of a wave works on the same chunk (the
  // appends are wave-wide); the chunk index is the wave-iteration index the
  // appends' regions and capacities are defined by.
  const unsigned n_chunks = (a.n + 63u) / 64u;
  const unsigned waves_per_block = blockDim.x / 64u;
  const unsigned W = gridDim.x * waves_per_block;
  const bool dyn_all = n_chunks >= 3u * W;            // every chunk from the counters
  const bool dyn_tail = !dyn_all && n_chunks > W;     // the first chunk static, the rest from the counters
  const bool dyn = dyn_all || dyn_tail;
  const unsigned X = gridDim.x < (unsigned)kChunkClasses ? gridDim.x : (unsigned)kChunkClasses;
  const unsigned cls = blockIdx.x % X;
  unsigned* ctr = a.cnt->chunk + ((size_t)a.g * kChunkClasses + cls) * kChunkStride;
  const unsigned c_base = dyn_all ? cls : W + cls;  // the class's k-th counter chunk: c_base + X k
  unsigned c = blockIdx.x * waves_per_block + threadIdx.x / 64u;
  if (dyn_all) {
    unsigned k0 = 0;
    if (lane_id() == 0) k0 = atomicAdd(ctr, 1u);
    c = cls + X * (unsigned)__shfl((int)k0, 0, 64);
  }
  // the chunk's rays, traversed: o, d and the hit of ray i (slot) of chunk c
  auto traverse = [&](unsigned i, bool valid, unsigned slot, V3& o, V3& d, Hit& h) {
    hit_init(h);
    if (valid) {
      wf_ray<CAM>(a, cam, slot, o, d);
      if constexpr (TALLY && QUADS) count_hier_gates(sc, o, d, t.gsk);
      if constexpr (LANE == 0) {
        // the chunk's frame (chunks never mix frames): its shared-origin primary records
        const unsigned pf = a.n_frames > 1 ? (c * 64u) / a.frame_rays : 0u;
        bvh_trace<PRIMARY, false>(sc, (cPrimRec)(a.prim + (size_t)pf * ((unsigned)sc.n_diag + 4)), stk, o, d, 0.0, h,
                                  t.disc, t.tests, t.boxes);
        trace_rest<false, QUADS, true>(sc, o, d, h, t.disc, &t.gsk);
        if constexpr (QUADS) {
          other_trace<false>(sc, o, d, 0.0, h, t.disc, t.tests, t.boxes);
          line_trace<false>(sc, o, d, 0.0, h, t.tests, t.boxes);
        }
      } else {
        // planes and the other records first: an early nearest hit tightens the culling
        trace_rest<false, QUADS, true>(sc, o, d, h, t.disc, &t.gsk);
        if constexpr (QUADS) {
          other_trace<false>(sc, o, d, 0.0, h, t.disc, t.tests, t.boxes);
          line_trace<false>(sc, o, d, 0.0, h, t.tests, t.boxes);
        }
        if constexpr (LANE == 14) {
          lane_trace_pair<false>(ls.nodes, ls.s48, ls.M, sc.n_bvh > 0, o, d, 0.0, h, t.disc, t.tests, t.boxes,
                                 ls.stack16);
        } else if constexpr (LANE == 15) {
          lane_trace_wide<false, Sph48, true>((const BvhWide*)ls.nodes, ls.s48, ls.M, sc.bvhw != nullptr, o, d, 0.0, h,
                                              t.disc, t.tests, t.boxes, ls.stack16, ls.wtop, ls.n_top, sc.n_diag);
        } else if constexpr (LANE == 4) {
          lane_trace_wide<false>((const BvhWide16*)ls.nodes, ls.sd, ls.M, sc.bvhw16 != nullptr, o, d, 0.0, h, t.disc,
                                 t.tests, t.boxes, ls.stack16, ls.wtop16, ls.n_top, sc.n_diag);
        } else {
          lane_trace<false, LANE == 3>((const BvhNode*)ls.nodes, ls.sd, ls.M, sc.n_bvh > 0, o, d, 0.0, h, t.disc,
                                       t.tests, t.boxes, ls.stack, ls.top, ls.n_top);
        }
      }
    }
    hit_finish(h);
  };
  while (c < n_chunks) {
    unsigned k_next = 0;
    if (dyn && lane_id() == 0) k_next = atomicAdd(ctr, 1u);
    const unsigned i = c * 64u + lane_id();
    // a batch's generation 0: the padding slots after each frame's root rays hold no ray
    const bool valid = i < a.n && (a.g != 0 || a.n_frames <= 1 || i % a.frame_rays < a.frame_real);
    const unsigned slot = valid ? shard_slot<true>(pre, a.in_cap, i) : 0u;
    V3 o = v3(0, 0, 0), d = v3(0, 0, 0);
    Hit h;
    traverse(i, valid, slot, o, d, h);
    shade_fused<LANE, QUADS, CAM>(sc, cam, a, ls, c, slot, valid, o, d, h, t);
    c = dyn ? c_base + X * (unsigned)__shfl((int)k_next, 0, 64) : c + W;
  }
  if constexpr (!TALLY) return;
  if (sc.n_groups) add_gate_skips(a.cnt, t.gsk);
  const unsigned long long s = wave_sum(t.disc), st = wave_sum(t.tests), sb = wave_sum(t.boxes);
  const unsigned long long hs = wave_sum(t.sh_disc), hst = wave_sum(t.sh_tests), hsb = wave_sum(t.sh_boxes);
  const unsigned long long hr = wave_sum(t.sh_rays);
  if (lane_id() == 0) {
    WfWorkRow* w = work_row(a.cnt);
    if (s) atomicAdd(&w->disc[a.disc_slot], s);
    if (st) atomicAdd(&w->tests[a.disc_slot], st);
    if (sb) atomicAdd(&w->boxes[a.disc_slot], sb);
    if (hs) atomicAdd(&w->disc[WF_SHADOW], hs);
    if (hst) { atomicAdd(&w->tests[WF_SHADOW], hst); atomicAdd(&w->sh_tests[a.disc_slot], hst); }
    if (hsb) atomicAdd(&w->boxes[WF_SHADOW], hsb);
    if (hr) atomicAdd(&w->sh_rays[a.disc_slot], hr);
  }
  if (a.count) {  // counted launch: shade_hit runs and children per generation (read_stats)
    const unsigned long long n1 = wave_sum(t.hits), n2 = wave_sum(t.refl), n3 = wave_sum(t.refr);
    if (lane_id() == 0) {
      if (n1) atomicAdd(&a.cnt->n_hit[a.g], (unsigned)n1);
      if (n2) atomicAdd(&a.cnt->n_refl[a.g], (unsigned)n2);
      if (n3) atomicAdd(&a.cnt->n_refr[a.g], (unsigned)n3);
    }
  }
}
#ifndef RT_WF_GLOBAL_TU
__global__ __launch_bounds__(kWfBlock) void wf_prep(DevScene sc, DevCamera cam, WfArgs a) {
  __shared__ unsigned s_pre[kPreRays];
  const unsigned* pre = shard_prefix<true>(a.in_cnt, s_pre);
  const unsigned stride = gridDim.x * blockDim.x;
  // every lane of a wave runs the same number of iterations (appends are wave-wide)
  const unsigned n_iter = (a.n + stride - 1) / stride;
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  for (unsigned it = 0; it < n_iter; ++it, i += stride) {
    const bool valid = i < a.n;
    const unsigned slot = valid ? shard_slot<true>(pre, a.in_cap, i) : 0u;
    V3 o = v3(0, 0, 0), d = v3(0, 0, 0);
    Hit h;
    h.key = -1;
    if (valid) {
      wf_ray(a, cam, slot, o, d);
      const WfHit w = a.hits[slot];
      h.t = w.t; h.key = w.key; h.hin = w.hin; h.c1k = w.c1k; h.c2k = w.c2k; h.c1t = 0; h.c2t = 0;
    }
    prep_one(sc, a, i, slot, valid, o, d, h);
  }
}

// ---------------------------------------------------------- combine
// World::shade_hit (world.rs:40-68) from the node, the shadow flags and the
// children's colours; color_at miss -> black (world.rs:74-75).
__global__ __launch_bounds__(kWfBlock) void wf_combine(DevScene sc, DevCamera cam, WfArgs a) {
  const unsigned stride = gridDim.x * blockDim.x;
  const unsigned L = (unsigned)sc.n_lights;
  __shared__ unsigned s_pre[kPreRays];
  const unsigned* pre = shard_prefix<true>(a.in_cnt, s_pre);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const unsigned slot = shard_slot<true>(pre, a.in_cap, i);
    const WfNode nd = a.nodes[slot];
    V3 color = v3(0.0, 0.0, 0.0);
    if (nd.obj >= 0) {
      const ShadeRec& m = sc.shade[nd.obj];
      V3 surface = v3(0.0, 0.0, 0.0);  // Sum = fold from (0,0,0) (color.rs:96-103)
      for (unsigned l = 0; l < L; ++l) {
        const double* sp = a.surf + ((size_t)slot * L + l) * 3;
        surface = vadd(surface, v3(sp[0], sp[1], sp[2]));
      }
      V3 refl = v3(0.0, 0.0, 0.0), refr = v3(0.0, 0.0, 0.0);
      if (nd.child_refl >= 0) {
        const double* cc = a.child_colors + (size_t)nd.child_refl * 3;
        refl = vscale(v3(cc[0], cc[1], cc[2]), m.reflective);  // world.rs:113
      }
      if (nd.child_refr >= 0) {
        const double* cc = a.child_colors + (size_t)nd.child_refr * 3;
        refr = vscale(v3(cc[0], cc[1], cc[2]), m.transparency);  // world.rs:133
      }
      if (m.reflective > 0.0 && m.transparency > 0.0) {
        const double r = nd.schlick;
        color = vadd(vadd(surface, vscale(refl, r)), vscale(refr, 1.0 - r));
      } else {
        color = vadd(vadd(surface, refl), refr);
      }
    }
    size_t oi = slot;
    if (a.g == 0 && a.camera_mode && a.aa == 1) {  // generation 0 is tile-ordered: write row-major
      uint32_t x, lr, smp;
      gen0_pixel(a.aa, a.rows, cam.hsize, i, x, lr, smp);
      oi = (size_t)lr * cam.hsize + x;
    }
    double* out = a.colors + oi * 3;
    out[0] = color.x; out[1] = color.y; out[2] = color.z;
  }
}

// The fast path's combine (DESIGN.md "Fused generations"): shade_hit of every
// node of generation g that has a reflected or refracted child, from its
// ParentRec (surface term, Schlick factor) and the children's colours, which
// generation g+1 wrote (directly or through this pass). Its parents' count
// comes from their region counters and their place from the generation table
// (device-sized generations). Generation 0's pass, the frame's last, also
// records the frame's ray count per generation in the workspace's host-mapped
// record (a.out_cnt: generation 1's ray counters), which sizes later frames.
// An asynchronous frame whose recursion outgrew the arenas (bind_generation)
// is incomplete, and it must never look valid in the caller's buffer (the
// reference's render never returns a partial canvas, camera.rs:133-148): the
// pass's last launch fills every canvas of the pass (each frame of a batch,
// `per_frame` outputs of 3 doubles) with NaN instead of colours. The call that
// finds the overflow (the next on the scene, or rt_scene_check) reports it;
// synchronous calls render such a frame again before they return.
__device__ __forceinline__ void poison_frames(const WfArgs& a, double* single, unsigned per_frame) {
  const unsigned nf = a.n_frames > 1 ? a.n_frames : 1u;
  const double nan = __builtin_nan("");
  const size_t n = (size_t)per_frame * 3, stride = (size_t)gridDim.x * blockDim.x;
  for (unsigned f = 0; f < nf; ++f) {
    double* o = a.n_frames > 1 ? a.frames->out[f] : single;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) o[i] = nan;
  }
}

__global__ __launch_bounds__(kWfBlock) void wf_combine_parents(DevScene sc, DevCamera cam, WfArgs a) {
  const unsigned stride = gridDim.x * blockDim.x;
  __shared__ unsigned s_pre[kPreList];
  const unsigned* pre = shard_prefix<false>(a.sh_cnt, s_pre);
  const WfGenTab t = a.gtab[a.g];
  const unsigned sh_cap = a.gsh[a.g];
  // (no room for the parents after an overflow: the counters hold what was asked for)
  const unsigned n = sh_cap ? (unsigned)__builtin_amdgcn_readfirstlane((int)pre[kShards]) : 0u;
  const ParentRec* parents = a.par_base + t.par_off;
  const double* child_colors = a.color_base + a.gtab[a.g + 1].color_off * 3ull;
  if (!(a.g == 0 && a.colors_direct)) a.colors = a.color_base + t.color_off * 3ull;
  if (a.g == 0 && blockIdx.x == 0 && threadIdx.x < 64) {
    volatile WfHostRec* r = a.hrec;
    for (unsigned l = threadIdx.x; l <= a.max_depth && l < (unsigned)kMaxGen; l += 64) {
      unsigned c = a.frame_real * (a.n_frames > 1 ? a.n_frames : 1u);
      if (l > 0) {
        const unsigned* q = a.out_cnt + (size_t)(l - 1) * 2 * kShards * kShardStride;
        c = 0;
        for (int k = 0; k < kShards; ++k) c += q[k * kShardStride] + q[k * kShardStride + 1];  // front + back
      }
      r->counts[l] = c;
    }
    if (threadIdx.x == 0) {
      r->n_real = a.frame_real * (a.n_frames > 1 ? a.n_frames : 1u);
      r->n_gens = a.max_depth + 1;
      r->frames = r->frames + 1;
    }
  }
  if (a.g == 0 && a.colors_direct && a.cnt->overflow) {  // (averaged frames: wf_average poisons them)
    poison_frames(a, a.colors, a.frame_real);
    return;
  }
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const ParentRec p = parents[shard_slot<false>(pre, sh_cap, i)];
    // the material's reflective and transparency values (the small per-object table)
    typedef double f64x2v __attribute__((ext_vector_type(2)));
    const f64x2v rt = *(const f64x2v*)(sc.refl_transp + 2 * (size_t)p.obj);
    V3 refl = v3(0.0, 0.0, 0.0), refr = v3(0.0, 0.0, 0.0);
    if (p.child_refl >= 0) {
      const double* cc = child_colors + (size_t)p.child_refl * 3;
      refl = vscale(v3(cc[0], cc[1], cc[2]), rt.x);  // world.rs:113
    }
    if (p.child_refr >= 0) {
      const double* cc = child_colors + (size_t)p.child_refr * 3;
      refr = vscale(v3(cc[0], cc[1], cc[2]), rt.y);  // world.rs:133
    }
    const V3 col = shade_color_rt(rt.x, rt.y, v3(p.surface[0], p.surface[1], p.surface[2]), refl, refr, p.schlick);
    double* out = color_dst(a, cam, p.slot);
    out[0] = col.x; out[1] = col.y; out[2] = col.z;
  }
}

// Color::average (color.rs:26-33) of the AA samples of each pixel: a left
// fold from black, then * (1 / n); written row-major (a batch: into each
// frame's canvas, its samples at that frame's generation-0 slots).
__global__ __launch_bounds__(kWfBlock) void wf_average(WfArgs a, unsigned hsize, const double* colors, unsigned n_pix,
                                                       double* out) {
  const unsigned stride = gridDim.x * blockDim.x;
  const unsigned aa = a.aa;
  const unsigned pix_frame = a.n_frames > 1 ? a.frame_real / aa : n_pix;
  if (a.cnt && a.cnt->overflow) {  // the fast path's pass outgrew its arenas: poison_frames
    poison_frames(a, out, pix_frame);
    return;
  }
  for (unsigned p = blockIdx.x * blockDim.x + threadIdx.x; p < n_pix; p += stride) {
    const unsigned f = p / pix_frame, lp = p - f * pix_frame;
    const size_t s0 = (size_t)f * (a.n_frames > 1 ? a.frame_rays : 0u) + (size_t)lp * aa;
    V3 sum = v3(0.0, 0.0, 0.0);
    for (unsigned s = 0; s < aa; ++s) {
      const double* c = colors + (s0 + s) * 3;
      sum = vadd(sum, v3(c[0], c[1], c[2]));
    }
    const V3 avg = vscale(sum, 1.0 / (double)aa);
    uint32_t x, lr, smp;
    gen0_pixel(a.aa, a.rows, hsize, lp * aa, x, lr, smp);
    double* o = (a.n_frames > 1 ? a.frames->out[f] : out) + ((size_t)lr * hsize + x) * 3;
    o[0] = avg.x; o[1] = avg.y; o[2] = avg.z;
  }
}

// Reflected / refracted ray counts per generation (stats only).
__global__ void wf_count_kinds(WfArgs a) {
  unsigned nrefl = 0, nrefr = 0, nhit = 0;
  const unsigned stride = gridDim.x * blockDim.x;
  __shared__ unsigned s_pre[kPreRays];
  const unsigned* pre = shard_prefix<true>(a.in_cnt, s_pre);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += stride) {
    const WfNode nd = a.nodes[shard_slot<true>(pre, a.in_cap, i)];
    nrefl += nd.child_refl >= 0;
    nrefr += nd.child_refr >= 0;
    nhit += nd.obj >= 0;  // shade_hit runs: one is_shadowed per light (world.rs:41-56)
  }
  const unsigned long long s1 = wave_sum(nrefl), s2 = wave_sum(nrefr), s3 = wave_sum(nhit);
  if (lane_id() == 0) {
    if (s1) atomicAdd(&a.cnt->n_refl[a.g], (unsigned)s1);
    if (s2) atomicAdd(&a.cnt->n_refr[a.g], (unsigned)s2);
    if (s3) atomicAdd(&a.cnt->n_hit[a.g], (unsigned)s3);
  }
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
  const int tb = trace_block(n, tn.adaptive_block);
  const size_t dl = a.use_lb ? delta_lds_bytes(sc) : 0;
  size_t dyn = 0;
  a.lds_flags = 0;
  // primary rays: the wave traversal, or with prim_lane the per-lane walk of the pair image or of
  // the four-wide hierarchy (the launches below, reading camera rays)
  const bool wide_ok = tn.image != 1 && tn.wide && sc.bvhw16 && wide_stack_bytes(sc) <= kWfLdsLimit / 2;
  // prim_lane 1: any per-lane image; 2 (default): the LDS images only (C3 primary class 0.128 ->
  // 0.125 ms/frame with the LDS four-wide image; C5's global image 2.06 -> 2.16 ms, so not there)
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

#else  // RT_WF_GLOBAL_TU
// The fast path's launches over the global-memory scene images (LANE 3: the
// treelet and the stack in LDS; LANE 1: the stack in LDS). This TU is the
// same source compiled a second time with -DRT_WF_GLOBAL_TU and without the
// AMDGPU register-pressure trackers (Makefile: rt_wavefront_glb.o), which
// help the LDS image (C3) and cost the global images (C5) ~2 %.
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
template <bool QUADS, int LANE, bool TALLY, bool CAM>
static hipError_t launch_glb(const DevScene& sc, const DevCamera& cam, const WfArgs& a, size_t dyn, unsigned n,
                             hipStream_t stream, int block, hipEvent_t e0, hipEvent_t e1) {
  auto kern = wf_trace_fused<false, QUADS, LANE, TALLY, CAM>;
  if (dyn > 0) WF_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
  const dim3 grid(occupancy_grid(kern, block, dyn, n));
  if (e0) hipExtLaunchKernelGGL(kern, grid, dim3(block), dyn, stream, e0, e1, 0, sc, cam, a);
  else hipLaunchKernelGGL(kern, grid, dim3(block), dyn, stream, sc, cam, a);
  return hipGetLastError();
}
template <int LANE>
static hipError_t launch_glb_lane(bool quads, bool tally, bool cam_rays, const DevScene& sc, const DevCamera& cam,
                                  const WfArgs& a, size_t dyn, unsigned n, hipStream_t stream, int block, hipEvent_t e0,
                                  hipEvent_t e1) {
#define RT_GLB(Q, T, C) launch_glb<Q, LANE, T, C>(sc, cam, a, dyn, n, stream, block, e0, e1)
  if (cam_rays) {
    if (quads) return tally ? RT_GLB(true, true, true) : RT_GLB(true, false, true);
    return tally ? RT_GLB(false, true, true) : RT_GLB(false, false, true);
  }
  if (quads) return tally ? RT_GLB(true, true, false) : RT_GLB(true, false, false);
  return tally ? RT_GLB(false, true, false) : RT_GLB(false, false, false);
#undef RT_GLB
}
hipError_t wf_launch_global(int lane, bool quads, bool tally, bool cam_rays, const DevScene& sc, const DevCamera& cam,
                            const WfArgs& a, size_t dyn, unsigned n, hipStream_t stream, int block, hipEvent_t e0,
                            hipEvent_t e1) {
  if (lane == 3) return launch_glb_lane<3>(quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, e0, e1);
  if (lane == 1) return launch_glb_lane<1>(quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, e0, e1);
  if (lane == 4) return launch_glb_lane<4>(quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, e0, e1);
  return hipErrorInvalidValue;
}
#endif  // RT_WF_GLOBAL_TU
}  // namespace rtamd
