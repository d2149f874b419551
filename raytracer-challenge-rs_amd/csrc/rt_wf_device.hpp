// rt_wf_device.hpp — the wavefront pipeline's device code shared by its
// translation units: queue appends and sharded slots, ray fetch, the LDS scene
// image, the trace loops and the fused generation kernel (wf_trace_fused:
// closest hit + shading + shadow rays + spawn). rt_wavefront.hip launches
// them over the LDS images, rt_wavefront_glb.hip over the global-memory
// images (its own code object); rt_wf_combine.hip holds the frame's other
// kernels (frame init, combine, average).
#pragma once
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
  // a hit on a sphere record: from inside, its shadow rays test that sphere first; from outside,
  // towards a light in front of the surface, they leave it out (shadow_trace)
  const int own = a.own_sphere ? sc.obj_diag[c.obj] : -1;
  const int own_first = own >= 0 && c.inside ? (own & kOwnIndex) : -1;
  const int own_out = own >= 0 && !c.inside && a.own_sphere > 1 && (own & kOwnOutside) ? (own & kOwnIndex) : -1;
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
                                                      t.sh_boxes, &t.gsk, own_first,
                                                      own_out >= 0 && vdot(sdir, c.normal) >= 0.0 ? own_out : -1);
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
  const unsigned n_chunks = (a.n + 63u) / 64u;
  const unsigned waves_per_block = blockDim.x / 64u;
  const unsigned W = gridDim.x * waves_per_block;
  // fewer chunks than waves (a small frame, a deep generation): chunk c goes to
  // block c mod grid, so that the chunks spread over every CU instead of filling
  // the first blocks' CUs (a block's waves share one CU: 16 latency-bound walks
  // on one CU against 4-5 each): a 320x240 frame alone 24-29 % faster, frames
  // in flight slower (WfTuning::spread, off by default; profiles/r06_spread.txt)
  const bool spread = a.spread && n_chunks < W;
  if (spread ? blockIdx.x >= n_chunks : blockIdx.x * waves_per_block >= n_chunks) return;
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
  const bool dyn_all = n_chunks >= 3u * W;            // every chunk from the counters
  const bool dyn_tail = !dyn_all && n_chunks > W;     // the first chunk static, the rest from the counters
  const bool dyn = dyn_all || dyn_tail;
  const unsigned X = gridDim.x < (unsigned)kChunkClasses ? gridDim.x : (unsigned)kChunkClasses;
  const unsigned cls = blockIdx.x % X;
  unsigned* ctr = a.cnt->chunk + ((size_t)a.g * kChunkClasses + cls) * kChunkStride;
  const unsigned c_base = dyn_all ? cls : W + cls;  // the class's k-th counter chunk: c_base + X k
  unsigned c = spread ? (threadIdx.x / 64u) * gridDim.x + blockIdx.x : blockIdx.x * waves_per_block + threadIdx.x / 64u;
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

// ---- the frame's other kernels (rt_wf_combine.hip), launched by rt_wavefront.hip
__global__ void wf_frame_init(DevScene sc, DevCamera cam, PrimRec* prim, unsigned do_prim, uint4* zero_a,
                              unsigned n_a, uint4* zero_b, unsigned n_b, FrameTable tab, FrameTable* tab_dev,
                              unsigned n_frames, WfGenTab* gtab);
__global__ void wf_prep(DevScene sc, DevCamera cam, WfArgs a);
__global__ void wf_combine(DevScene sc, DevCamera cam, WfArgs a);
__global__ void wf_combine_parents(DevScene sc, DevCamera cam, WfArgs a);
__global__ void wf_average(WfArgs a, unsigned hsize, const double* colors, unsigned n_pix, double* out);
__global__ void wf_count_kinds(WfArgs a);

}  // namespace rtamd
