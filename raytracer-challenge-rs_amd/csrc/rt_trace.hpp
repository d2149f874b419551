// rt_trace.hpp — device-side traversal and shading pieces of the generation
// pipeline (rt_wavefront.hip): the exact-culling BVH traversals, the
// light-buffer shadow walk, the per-block LDS scene image, and the small
// shading helpers. Include only from .hip files compiled with
// -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rt_device.hpp"
#include "rt_wavefront.hpp"

#pragma clang fp contract(off)

namespace rtamd {

constexpr int kTraceBlock = 1024;  // trace kernels: 16 waves, one LDS image per block

__device__ __forceinline__ unsigned lane_id() { return __lane_id(); }

// AA sample offsets of Camera::get_offsets (camera.rs:92-126), per count
// 1, 2, 4, 8, 16 at offsets 0, 1, 3, 7, 15 of the table.
static __constant__ double kAaOffsets[31][2] = {
    {0.5, 0.5},
    {0.25, 0.5}, {0.75, 0.5},
    {0.25, 0.25}, {0.75, 0.25}, {0.25, 0.75}, {0.75, 0.75},
    {0.25, 0.25}, {0.5, 0.25}, {0.75, 0.25}, {0.25, 0.5}, {0.75, 0.5}, {0.25, 0.75}, {0.5, 0.75}, {0.75, 0.75},
    {0.125, 0.125}, {0.375, 0.125}, {0.625, 0.125}, {0.875, 0.125},
    {0.125, 0.375}, {0.375, 0.375}, {0.625, 0.375}, {0.875, 0.375},
    {0.125, 0.625}, {0.375, 0.625}, {0.625, 0.625}, {0.875, 0.625},
    {0.125, 0.875}, {0.375, 0.875}, {0.625, 0.875}, {0.875, 0.875}};

// Generation-0 ray order of a camera shard: the shard's local rows in bands
// of 8, each band in tiles of 8 columns, AA samples innermost, so one wave
// holds an 8x8 pixel tile (coherent rays for the BVH traversal). Returns the
// pixel (x, local row) and the sample index of ray i.
__device__ __forceinline__ void gen0_pixel(uint32_t aa, uint32_t rows, uint32_t hsize, uint32_t i, uint32_t& x, uint32_t& lr,
                                           uint32_t& smp) {
  const uint32_t p = i / aa;
  smp = i - p * aa;
  const uint32_t band = p / (8u * hsize);
  const uint32_t r0 = band * 8u;
  const uint32_t R = min(8u, rows - r0);
  const uint32_t j = p - band * 8u * hsize;
  const uint32_t t = j / (8u * R);
  const uint32_t w = min(8u, hsize - 8u * t);
  const uint32_t within = j - t * 8u * R;
  const uint32_t wy = within / w;
  x = 8u * t + (within - wy * w);
  lr = r0 + wy;
}

// A shadow ray whose answer cannot change the colour (DESIGN.md "Skipped
// shadow rays"): with the light behind the surface, lighting() returns
// `ambient` in shadow and `ambient + 0 + 0` in light (material.rs:23-87),
// bit-identical unless a component of ambient is -0 or NaN. Evaluated with
// the operations lighting() itself performs; patterned materials are never
// skipped. Returns whether it is, and that ambient value.
// `lightv` = (light.position - over).normalize(), the shadow ray's direction.
__device__ __forceinline__ bool shadow_irrelevant(const ShadeRec& m, cLightRec L, V3 lightv, V3 normal, V3& ambient) {
  if (m.pattern_kind >= 0) return false;
  if (!(vdot(lightv, normal) < 0.0)) return false;
  const V3 effective_color = vmul(v3(m.color[0], m.color[1], m.color[2]),
                                  v3(L->intensity[0], L->intensity[1], L->intensity[2]));
  ambient = vscale(effective_color, m.ambient);
  auto plain = [](double x) { return x == x && !(x == 0.0 && signbit(x)); };
  return plain(ambient.x) && plain(ambient.y) && plain(ambient.z);
}

// ------------------------------------------------------------ BVH traversal
// Exact culling (DESIGN.md "Exact culling"): the wave traverses the sphere
// BVH together (wave-uniform stack in LDS, wave-uniform 64-B node loads) and
// skips a child only when NO lane's ray meets its padded box within
// [0, t_hi] (t_hi = the lane's current nearest hit, or the light distance for
// shadow rays). A sphere the exhaustive loop would hit always lies in a box
// that passes, and the per-lane results are order-independent minima, so the
// results are bit-identical to the exhaustive loop. Lanes whose rays miss a
// visited leaf still test its spheres (harmless: exhaustive work).
typedef const RT_CONST BvhNode* cBvhNode;
typedef const RT_CONST PrimRec* cPrimRec;

// The per-lane traversal's slab test runs in binary32 on an interval that is
// widened to contain the exact (real-arithmetic) one; DESIGN.md §5.2 has the
// error bound. Per ray and axis: inv = an approximate reciprocal of d in
// binary32 (slab_inv: relative error below 2^-22, exactly the value the FMAs
// use), and the plane constants c = o*inv -/+ delta with delta = 2^-20 |inv|
// (M + |o|), where M bounds every box coordinate on that axis (the root's
// children); the computed entry (exit) distance fma(corner, inv, -c) then
// never exceeds (falls short of) the exact one, (corner - o) / d: its error,
// the reciprocal's included, is below delta/3.
// An axis whose direction is (nearly) zero or whose origin is huge / NaN is
// not used for culling at all (interval (-inf, +inf)).
struct SlabRay {
  float inv[3], c_lo[3], c_hi[3];
};
// binary32 reciprocal of a binary64 direction component with 2^-60 <= |d|:
// (float)d rounds once (2^-24), v_rcp_f32 is within 1 ulp (2^-23); returned
// widened to binary64 (exact), the value every plane constant is built from.
__device__ __forceinline__ double slab_inv(double d) { return (double)__builtin_amdgcn_rcpf((float)d); }
__device__ __forceinline__ SlabRay slab_ray(V3 o, V3 d, const float* M) {
  SlabRay r;
  const double oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (fabs(da[a]) >= 0x1p-60 && fabs(oa[a]) <= 0x1p60 && M[a] <= 0x1p60f) {  // NaN fails
      const double inv = slab_inv(da[a]);
      const double oinv = oa[a] * inv;
      const double delta = 0x1p-20 * fabs(inv) * ((double)M[a] + fabs(oa[a]));
      const float on = (float)(oinv + delta), of = (float)(oinv - delta);
      r.inv[a] = (float)inv;
      r.c_lo[a] = inv >= 0.0 ? on : of;  // the lo plane is the entry plane when inv >= 0
      r.c_hi[a] = inv >= 0.0 ? of : on;
    } else {
      r.inv[a] = 0.0f;
      r.c_lo[a] = INFINITY;
      r.c_hi[a] = -INFINITY;
    }
  }
  return r;
}
// binary32 upper bound of a non-negative binary64 distance: RN(x) is within
// 2^-23 of x relative to it, and RN(f * (1 + 2^-22)) > f * (1 + 2^-23)
// (0 and inf map to themselves).
__device__ __forceinline__ float f32_up(double x) { return (float)x * (1.0f + 0x1p-22f); }
// max(entry, 0) <= min(exit, t_hi): the ray may meet the box within [0, t_hi]
// (t_hi >= 0). `t_in` = the widened entry distance (child ordering only).
template <typename P>  // P: constant-address (scalar loads) or generic (per-lane loads) float pointer
__device__ __forceinline__ bool slab_hit32(P lo, P hi, const SlabRay& r, float t_hi, float& t_in) {
  const float x0 = fmaf(lo[0], r.inv[0], -r.c_lo[0]), x1 = fmaf(hi[0], r.inv[0], -r.c_hi[0]);
  const float y0 = fmaf(lo[1], r.inv[1], -r.c_lo[1]), y1 = fmaf(hi[1], r.inv[1], -r.c_hi[1]);
  const float z0 = fmaf(lo[2], r.inv[2], -r.c_lo[2]), z1 = fmaf(hi[2], r.inv[2], -r.c_hi[2]);
  const float tmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
  const float tmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t_hi));
  t_in = tmin;
  return tmin <= tmax;
}

template <bool PRIMARY, bool SHADOW>
__device__ __forceinline__ void bvh_trace(const DevScene& sc, cPrimRec prim, int* stk, V3 o, V3 d, double t_shadow,
                                          Hit& h, unsigned& n_disc, unsigned& n_tests, unsigned& n_boxes) {
  hit_init(h);
  const cBvhNode nodes = (cBvhNode)sc.bvh;
  float M[3];
  for (int a = 0; a < 3; ++a)
    M[a] = fmaxf(fmaxf(fabsf(nodes->lo[0][a]), fabsf(nodes->hi[0][a])),
                 fmaxf(fabsf(nodes->lo[1][a]), fabsf(nodes->hi[1][a])));
  const SlabRay sr = slab_ray(o, d, M);
  const float t_sh = SHADOW ? f32_up(t_shadow) : 0.0f;
  const cSphereDiag sd = (cSphereDiag)sc.sph_diag;
  int sp = 1;
  stk[0] = 0;
  while (sp > 0) {
    --sp;
    const int e = __builtin_amdgcn_readfirstlane(stk[sp]);
    if (e < 0) {  // leaf: first << 7 | count
      const int code = -(e + 1);
      const int first = code >> 7, cnt = code & 127;
      for (int k = first; k < first + cnt; ++k) {
        if constexpr (PRIMARY) {
          const cPrimRec r = prim + k;
          const double dx = r->s[0] * d.x, dy = r->s[1] * d.y, dz = r->s[2] * d.z;
          sphere_adc<false>(dx * dx + dy * dy + dz * dz, dx * r->op[0] + dy * r->op[1] + dz * r->op[2], r->c,
                            [&] { return (int)sd[k].meta; }, h, n_disc);
        } else {
          diag_test<SHADOW>(sd + k, o, d, h, n_disc);
        }
      }
      n_tests += (unsigned)cnt;
      if constexpr (SHADOW) {
        if (!__any(!(h.key >= 0 && h.t < t_shadow))) break;  // every lane is shadowed
      }
      continue;
    }
    const cBvhNode nd = nodes + e;
    const float t_hi = SHADOW ? t_sh : f32_up(h.t);
    const int c0 = nd->child[0], c1 = nd->child[1];
    float t0, t1;
    const bool h0 = slab_hit32(nd->lo[0], nd->hi[0], sr, t_hi, t0);
    const bool h1 = c1 != kBvhEmpty && slab_hit32(nd->lo[1], nd->hi[1], sr, t_hi, t1);
    n_boxes += 2;
    const bool any0 = __any(h0), any1 = __any(h1);
    // push the far child first so the near one (by the lead lane's direction) pops first
    const int axis = nd->axis;
    const double dax = axis == 0 ? d.x : axis == 1 ? d.y : d.z;
    const bool flip = __builtin_amdgcn_readfirstlane(dax < 0.0 ? 1 : 0) != 0;
    const int near_c = flip ? c1 : c0, far_c = flip ? c0 : c1;
    const bool near_hit = flip ? any1 : any0, far_hit = flip ? any0 : any1;
    if (far_hit) stk[sp++] = far_c;
    if (near_hit) stk[sp++] = near_c;
  }
}

// Per-lane traversal for incoherent rays (secondary and shadow generations)
// over the binary node layout in global memory (scenes whose image does not
// fit in LDS): every lane walks the BVH on its own (near child first by its
// own direction, a private stack), so a wave pays for the longest path
// instead of the union of 64 paths. Same culling rule and the same exactness
// argument as the wave traversal above.
// LDS_STACK: the stack lives in LDS, entry k of lane t at lds[k * kTraceBlock + t]
// (needs bvh_depth <= kLaneLdsDepth); otherwise in private (scratch) memory.
// `h` arrives initialised (it may already hold the planes' nearest hit, which
// tightens the culling).
__device__ __forceinline__ void node_chunks(const BvhNode* nodes, int e, uint4& q0, uint4& q1, uint4& q2, uint4& q3) {
  const uint4* b = reinterpret_cast<const uint4*>(nodes);
  q0 = b[4 * e]; q1 = b[4 * e + 1]; q2 = b[4 * e + 2]; q3 = b[4 * e + 3];
}
template <bool SHADOW>
__device__ __forceinline__ void leaf_sphere_test(const SphereDiag* sd, int k, V3 o, V3 d, Hit& h, unsigned& n_disc) {
  const SphereDiag& r = sd[k];
  const double s0 = r.s[0], s1 = r.s[1], s2 = r.s[2];
  sphere_test<SHADOW>(s0 * o.x + r.t[0], s1 * o.y + r.t[1], s2 * o.z + r.t[2], s0 * d.x, s1 * d.y, s2 * d.z,
                      [&] { return (int)r.meta; }, h, n_disc);
}
// The pair image's LDS copy of the sphere records (lane_scene, LANE 14): 48 B
// per record (s[3], t[3]) and the metas apart, 52 B instead of 64.
struct Sph48 {
  const double* r;   // 6 doubles per record
  const int* meta;
};
template <bool SHADOW>
__device__ __forceinline__ void leaf_sphere_test(Sph48 sd, int k, V3 o, V3 d, Hit& h, unsigned& n_disc) {
  const double* r = sd.r + 6 * k;
  const double s0 = r[0], s1 = r[1], s2 = r[2];
  sphere_test<SHADOW>(s0 * o.x + r[3], s1 * o.y + r[4], s2 * o.z + r[5], s0 * d.x, s1 * d.y, s2 * d.z,
                      [&] { return sd.meta[k]; }, h, n_disc);
}

// With a treelet (the global-memory image), the first n_top nodes (breadth-first:
// the top levels) are read from their LDS copy `top`, the rest from `nodes`.
template <bool SHADOW, bool LDS_STACK>
__device__ __forceinline__ void lane_trace(const BvhNode* nodes, const SphereDiag* sd, const float* M, bool has_bvh,
                                           V3 o, V3 d, double t_shadow, Hit& h, unsigned& n_disc, unsigned& n_tests,
                                           unsigned& n_boxes, int* lds, const BvhNode* top = nullptr,
                                           int n_top = 0) {
  const SlabRay sr = slab_ray(o, d, M);
  float t_hi = f32_up(SHADOW ? t_shadow : h.t);
  int pstk[LDS_STACK ? 1 : kBvhMaxDepth + 4];
  auto stk = [&](int k) -> int& { if constexpr (LDS_STACK) return lds[k * kTraceBlock]; else return pstk[k]; };
  int sp = 0;
  auto pop = [&]() { return sp > 0 ? stk(--sp) : kBvhEmpty; };
  int e = (SHADOW && h.key >= 0 && h.t < t_shadow) || !has_bvh ? kBvhEmpty : 0;
  // a node visit: both children's boxes, the one entered first visited first
  auto visit = [&]() {
    // the whole 64-B node in four 16-B loads: lo[0], lo[1], hi[0], hi[1], child[2], axis, pad
    // (explicit address spaces: the two paths stay LDS and global loads)
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 r0, r1, r2, r3;
    if (e < n_top) {
      typedef __attribute__((address_space(3))) const u32x4 lq;
      lq* b = (lq*)(top + e);
      r0 = b[0]; r1 = b[1]; r2 = b[2]; r3 = b[3];
    } else {
      typedef __attribute__((address_space(1))) const u32x4 gq;
      gq* b = (gq*)(nodes + e);
      r0 = b[0]; r1 = b[1]; r2 = b[2]; r3 = b[3];
    }
    const uint4 q0 = make_uint4(r0.x, r0.y, r0.z, r0.w), q1 = make_uint4(r1.x, r1.y, r1.z, r1.w);
    const uint4 q2 = make_uint4(r2.x, r2.y, r2.z, r2.w), q3 = make_uint4(r3.x, r3.y, r3.z, r3.w);
    const float lo0[3] = {__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z)};
    const float lo1[3] = {__uint_as_float(q0.w), __uint_as_float(q1.x), __uint_as_float(q1.y)};
    const float hi0[3] = {__uint_as_float(q1.z), __uint_as_float(q1.w), __uint_as_float(q2.x)};
    const float hi1[3] = {__uint_as_float(q2.y), __uint_as_float(q2.z), __uint_as_float(q2.w)};
    const int c0 = (int)q3.x, c1 = (int)q3.y;
    float t0, t1;
    const bool h0 = slab_hit32(lo0, hi0, sr, t_hi, t0);
    const bool h1 = slab_hit32(lo1, hi1, sr, t_hi, t1) & (c1 != kBvhEmpty);
    n_boxes += 2;
    if (h0 && h1) {
      const bool flip = t1 < t0;
      stk(sp++) = flip ? c0 : c1;
      e = flip ? c1 : c0;
    } else {
      e = h0 ? c0 : h1 ? c1 : pop();
    }
  };
  // a leaf's spheres; true when a shadow ray is found occluded
  auto leaf = [&](int code_e) {
    const int code = -(code_e + 1);
    const int first = code >> 7, cnt = code & 127;
    for (int k = first; k < first + cnt; ++k) leaf_sphere_test<SHADOW>(sd, k, o, d, h, n_disc);
    n_tests += (unsigned)cnt;
    if constexpr (SHADOW) {
      return h.key >= 0 && h.t < t_shadow;
    } else {
      t_hi = f32_up(h.t);
      return false;
    }
  };
  // Leaves batched across the wave (speculative while-while): a lane meeting
  // a leaf postpones it and keeps visiting nodes; the node phase ends when no
  // lane without a postponed leaf has a node left, then all postponed leaves
  // are tested together. Culling only ever uses the lane's current bound, so
  // the postponement changes no result.
  int pl = kBvhEmpty;
  for (;;) {
    for (;;) {
      if (e < 0 && e != kBvhEmpty && pl == kBvhEmpty) { pl = e; e = pop(); }
      if (!__any(e >= 0 && pl == kBvhEmpty)) break;
      if (e >= 0) visit();  // lanes holding a leaf keep going (speculative)
    }
    if (!__any(pl != kBvhEmpty)) break;
    if (pl != kBvhEmpty) {
      if (leaf(pl)) { e = kBvhEmpty; sp = 0; }  // shadowed: done
      pl = kBvhEmpty;
    }
  }
}
// Per-lane traversal over the four-wide layout (NODE: BvhWide, 128-B binary32
// nodes, LANE 15 with the whole image in LDS; BvhWide16, 64-B binary16 nodes,
// LANE 4 from global memory with a treelet in LDS): a visit loads the parts of
// the node it needs (per axis the block of the four entry planes and the block
// of the four exit planes, chosen by the sign of the ray's direction there as
// in lane_trace_pair, whose byte offsets sit packed in two registers: six 16-B
// loads, or six 8-B ones for binary16; and the four child codes in one 8-B
// load), tests the four boxes with no per-axis min/max, goes on to the nearest
// child hit and pushes the others farthest first. The order is a sorting
// network over four 32-bit keys (the entry distance's bits with the slot in
// the two low bits, a miss all ones: non-negative binary32 values order as
// their bits do; ties and the two dropped bits only change the visit order);
// the slots' child codes come from one 64-bit word. A ray makes about half the
// dependent node loads of the binary walk. The stack is 16-bit, in LDS (entry
// k of lane t at lds[k * kTraceBlock + t], sc.bvhw_stack entries at most); the
// first n_top nodes are read from their LDS copy `top`. Culling is
// slab_hit32's rule (the same entry and exit values) on boxes that each hold
// what lies below them, so the hit is the same. Binary16 planes enter the
// binary32 FMA exactly (v_fma_mix_f32); since their outward rounding moves a
// coordinate by up to 2^-10 of its magnitude, slab_ray's bound M is widened by
// 2^-9 of itself for them (an infinite plane, past binary16's range, gives an
// infinite distance, or NaN on an axis that culls nothing, which the min/max
// drop). Empty slots have inverted boxes, which cull themselves for every ray
// with a usable axis, and a ray with none (a huge origin, a NaN) tests every
// record, as a walk that culls nothing would. Leaves are batched across the
// wave as in lane_trace.
// SD: the sphere records (const SphereDiag* in global memory, or Sph48 in LDS);
// ALL_LDS: every node is in `top` (LANE 15: the whole hierarchy in LDS).
template <bool SHADOW, typename SD = const SphereDiag*, bool ALL_LDS = false, typename NODE = BvhWide>
__device__ __forceinline__ void lane_trace_wide(const NODE* nodes, SD sd, const float* M,
                                                bool has_bvh, V3 o, V3 d, double t_shadow, Hit& h, unsigned& n_disc,
                                                unsigned& n_tests, unsigned& n_boxes, uint16_t* lds,
                                                const NODE* top, int n_top, int n_records) {
  constexpr bool H = sizeof(NODE) == 64;  // BvhWide16
  constexpr unsigned kBlk = H ? 8u : 16u, kHi = 3u * kBlk, kCc = 6u * kBlk;  // plane block, hi planes, child codes
  const float w = H ? 1.0f + 0x1p-9f : 1.0f;
  const float Mw[3] = {M[0] * w, M[1] * w, M[2] * w};
  const SlabRay sr = slab_ray(o, d, Mw);
  float t_hi = f32_up(SHADOW ? t_shadow : h.t);
  int sp = 0;
  auto pop = [&]() -> unsigned { return sp > 0 ? (unsigned)lds[(--sp) * kTraceBlock] : kWideEmpty; };
  unsigned e = (SHADOW && h.key >= 0 && h.t < t_shadow) || !has_bvh ? kWideEmpty : 0u;
  // per axis the entry planes' block (lo[a] when inv >= 0, else hi[a]) with the
  // constant `on`, the exit block with `of`
  float on[3], of[3];
  unsigned offe = 0, offx = 0;
  bool usable = false;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const bool neg = sr.inv[a] < 0.0f;
    on[a] = neg ? sr.c_hi[a] : sr.c_lo[a];
    of[a] = neg ? sr.c_lo[a] : sr.c_hi[a];
    usable |= sr.inv[a] != 0.0f;
    offe |= (kBlk * a + (neg ? kHi : 0u)) << (8 * a);
    offx |= (kBlk * a + (neg ? 0u : kHi)) << (8 * a);
  }
  asm volatile("" : "+v"(offe), "+v"(offx));
  if (e == 0u && !usable) {  // no axis can cull (empty slots' inverted boxes need one): every record
    e = kWideEmpty;
    for (int k = 0; k < n_records; ++k) {
      leaf_sphere_test<SHADOW>(sd, k, o, d, h, n_disc);
      ++n_tests;
      if (SHADOW && h.key >= 0 && h.t < t_shadow) break;
    }
  }
  auto visit = [&]() {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef typename std::conditional<H, u32x2, u32x4>::type Blk;  // one block of four planes
    Blk E[3], X[3];
    u32x2 cc;
    if (ALL_LDS || (int)e < n_top) {
      typedef __attribute__((address_space(3))) const unsigned char lb;
      lb* b = (lb*)(top) + e * (unsigned)sizeof(NODE);
      cc = *(__attribute__((address_space(3))) const u32x2*)(b + kCc);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        E[a] = *(__attribute__((address_space(3))) const Blk*)(b + ((offe >> (8 * a)) & 0xFFu));
        X[a] = *(__attribute__((address_space(3))) const Blk*)(b + ((offx >> (8 * a)) & 0xFFu));
      }
    } else {
      typedef __attribute__((address_space(1))) const unsigned char gb;
      gb* b = (gb*)(nodes);
      const unsigned n0 = e * (unsigned)sizeof(NODE);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        E[a] = *(__attribute__((address_space(1))) const Blk*)(b + (n0 + ((offe >> (8 * a)) & 0xFFu)));
        X[a] = *(__attribute__((address_space(1))) const Blk*)(b + (n0 + ((offx >> (8 * a)) & 0xFFu)));
      }
      cc = *(__attribute__((address_space(1))) const u32x2*)(b + (n0 + kCc));
    }
    // plane j of a block (binary16: converted inside the FMA, v_fma_mix_f32)
    auto pl = [&](const Blk& q, int j) -> float {
      if constexpr (H) return (float)__builtin_bit_cast(f16x4, q)[j];
      else return __uint_as_float(q[j]);
    };
    unsigned key[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t0 = fmaxf(fmaxf(fmaf(pl(E[0], j), sr.inv[0], -on[0]), fmaf(pl(E[1], j), sr.inv[1], -on[1])),
                             fmaxf(fmaf(pl(E[2], j), sr.inv[2], -on[2]), 0.0f));
      float zt;  // (t_hi is canonical: no per-visit re-canonicalisation, as in lane_trace_pair)
      asm("v_min_f32 %0, %1, %2" : "=v"(zt) : "v"(fmaf(pl(X[2], j), sr.inv[2], -of[2])), "v"(t_hi));
      const float t1 = fminf(fminf(fmaf(pl(X[0], j), sr.inv[0], -of[0]), fmaf(pl(X[1], j), sr.inv[1], -of[1])), zt);
      key[j] = t0 <= t1 ? ((__float_as_uint(t0) & ~3u) | (unsigned)j) : ~0u;
    }
    n_boxes += 4;
    auto cx = [&](int a, int b) {
      const unsigned lo = min(key[a], key[b]), hi = max(key[a], key[b]);
      key[a] = lo;
      key[b] = hi;
    };
    cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
    const unsigned long long P = ((unsigned long long)cc.y << 32) | cc.x;
    auto child = [&](unsigned k) { return (unsigned)(P >> ((k & 3u) << 4)); };  // (low 16 bits)
    if (key[3] != ~0u) lds[(sp++) * kTraceBlock] = (uint16_t)child(key[3]);
    if (key[2] != ~0u) lds[(sp++) * kTraceBlock] = (uint16_t)child(key[2]);
    if (key[1] != ~0u) lds[(sp++) * kTraceBlock] = (uint16_t)child(key[1]);
    e = key[0] != ~0u ? (child(key[0]) & 0xFFFFu) : pop();
  };
  // a leaf's record; true when a shadow ray is found occluded
  auto leaf = [&](unsigned code) {
    leaf_sphere_test<SHADOW>(sd, (int)(code & 0x7FFFu), o, d, h, n_disc);
    ++n_tests;
    if constexpr (SHADOW) {
      return h.key >= 0 && h.t < t_shadow;
    } else {
      t_hi = f32_up(h.t);
      return false;
    }
  };
  // leaves batched across the wave, as lane_trace does
  unsigned pl = kWideEmpty;
  for (;;) {
    for (;;) {
      if (e >= kWideLeaf && e != kWideEmpty && pl == kWideEmpty) { pl = e; e = pop(); }
      if (!__any(e < kWideLeaf && pl == kWideEmpty)) break;
      if (e < kWideLeaf) visit();  // lanes holding a leaf keep going (speculative)
    }
    if (!__any(pl != kWideEmpty)) break;
    if (pl != kWideEmpty) {
      if (leaf(pl)) { e = kWideEmpty; sp = 0; }  // shadowed: done
      pl = kWideEmpty;
    }
  }
}

// Per-lane traversal over the pair layout (LANE == 14): the block's LDS copy
// of each binary node stores, per axis, the two children's lower bounds as
// one 8-B pair and their upper bounds as the next pair (lo0 lo1 hi0 hi1 per
// axis, then the child codes). Which face a ray enters on an axis follows the
// sign of its direction there, so each lane computes once the byte offsets of
// its entry and exit pairs and loads them directly: one packed binary32 FMA
// gives both children's entry (or exit) distances on an axis, and no per-axis
// min/max is needed to tell entry from exit. The entry and exit values are the
// ones lane_trace computes (entry = fma(entry face, inv, -on), exit =
// fma(exit face, inv, -of), where lane_trace's min/max picks exactly them), so
// the culling and the visit order are the same bit for bit. Leaves are
// batched across the wave as in lane_trace<..., WW>.
// The pair image's child codes are 16-bit (rt_layout.hpp BvhPair: a node
// index below 0x8000, a leaf 0x8000 | first << 3 | (count - 1), 0xFFFF
// empty), so the per-lane LDS stack holds 16-bit entries.
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kPairEmpty = 0xFFFF;
template <bool SHADOW>
__device__ __forceinline__ void lane_trace_pair(const unsigned char* nodes, Sph48 sd, const float* M,
                                                bool has_bvh, V3 o, V3 d, double t_shadow, Hit& h, unsigned& n_disc,
                                                unsigned& n_tests, unsigned& n_boxes, uint16_t* lds) {
  float inv[3], on[3], of[3];
  int ent[3], ext[3];
  {
    const double oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      bool neg = false;
      if (fabs(da[a]) >= 0x1p-60 && fabs(oa[a]) <= 0x1p60 && M[a] <= 0x1p60f) {  // as slab_ray; NaN fails
        const double iv = slab_inv(da[a]);
        const double oinv = oa[a] * iv;
        const double delta = 0x1p-20 * fabs(iv) * ((double)M[a] + fabs(oa[a]));
        inv[a] = (float)iv;
        on[a] = (float)(oinv + delta);
        of[a] = (float)(oinv - delta);
        neg = !(iv >= 0.0);
      } else {
        inv[a] = 0.0f;
        on[a] = INFINITY;
        of[a] = -INFINITY;
      }
      ent[a] = 16 * a + (neg ? 8 : 0);
      ext[a] = ent[a] ^ 8;
    }
  }
  // keep the six offsets in registers (the compiler would otherwise recompute
  // the exit offsets in every visit)
#pragma unroll
  for (int a = 0; a < 3; ++a) asm volatile("" : "+v"(ent[a]), "+v"(ext[a]));
  float t_hi = f32_up(SHADOW ? t_shadow : h.t);
  auto stk = [&](int k) -> uint16_t& { return lds[k * kTraceBlock]; };
  // entry 0 is a sentinel (kPairEmpty): a pop needs no emptiness test, and a
  // lane that pops it is done and pops no more (the stack holds bvh_depth + 1)
  stk(0) = (uint16_t)kPairEmpty;
  int sp = 1;
  auto pop = [&]() { return (int)stk(--sp); };
  int e = (SHADOW && h.key >= 0 && h.t < t_shadow) || !has_bvh ? kPairEmpty : 0;
  auto visit = [&]() {
    const unsigned char* nb = nodes + (size_t)e * 64;
    const f32x2 ex = *(const f32x2*)(nb + ent[0]), ey = *(const f32x2*)(nb + ent[1]), ez = *(const f32x2*)(nb + ent[2]);
    const f32x2 xx = *(const f32x2*)(nb + ext[0]), xy = *(const f32x2*)(nb + ext[1]), xz = *(const f32x2*)(nb + ext[2]);
    const int2 cc = *(const int2*)(nb + 48);
    const f32x2 tx0 = __builtin_elementwise_fma(ex, (f32x2)(inv[0]), (f32x2)(-on[0]));
    const f32x2 ty0 = __builtin_elementwise_fma(ey, (f32x2)(inv[1]), (f32x2)(-on[1]));
    const f32x2 tz0 = __builtin_elementwise_fma(ez, (f32x2)(inv[2]), (f32x2)(-on[2]));
    const f32x2 tx1 = __builtin_elementwise_fma(xx, (f32x2)(inv[0]), (f32x2)(-of[0]));
    const f32x2 ty1 = __builtin_elementwise_fma(xy, (f32x2)(inv[1]), (f32x2)(-of[1]));
    const f32x2 tz1 = __builtin_elementwise_fma(xz, (f32x2)(inv[2]), (f32x2)(-of[2]));
    const float t0 = fmaxf(fmaxf(tx0.x, ty0.x), fmaxf(tz0.x, 0.0f));
    const float t1 = fmaxf(fmaxf(tx0.y, ty0.y), fmaxf(tz0.y, 0.0f));
    // (t_hi is canonical already: a v_min_f32 of our own keeps the compiler from
    // re-canonicalising it in every visit; C3 closest class 0.866 -> 0.857 ms)
    float zt0, zt1;
    asm("v_min_f32 %0, %1, %2" : "=v"(zt0) : "v"(tz1.x), "v"(t_hi));
    asm("v_min_f32 %0, %1, %2" : "=v"(zt1) : "v"(tz1.y), "v"(t_hi));
    const float u0 = fminf(fminf(tx1.x, ty1.x), zt0);
    const float u1 = fminf(fminf(tx1.y, ty1.y), zt1);
    const bool h0 = t0 <= u0;
    const bool h1 = (t1 <= u1) & (cc.y != kPairEmpty);
    n_boxes += 2;
    if (h0 && h1) {
      const bool flip = t1 < t0;
      stk(sp++) = (uint16_t)(flip ? cc.x : cc.y);
      e = flip ? cc.y : cc.x;
    } else {
      e = h0 ? cc.x : h1 ? cc.y : pop();
    }
  };
  auto leaf = [&](int code) {
    const int first = (code >> 3) & 0xFFF, cnt = (code & 7) + 1;
    for (int k = first; k < first + cnt; ++k) leaf_sphere_test<SHADOW>(sd, k, o, d, h, n_disc);
    n_tests += (unsigned)cnt;
    if constexpr (SHADOW) {
      return h.key >= 0 && h.t < t_shadow;
    } else {
      t_hi = f32_up(h.t);
      return false;
    }
  };
  int pl = kPairEmpty;
  for (;;) {
    for (;;) {
      if (e >= 0x8000 && e != kPairEmpty && pl == kPairEmpty) { pl = e; e = pop(); }
      if (!__any(e < 0x8000 && pl == kPairEmpty)) break;
      if (e < 0x8000) visit();  // lanes holding a leaf keep going (speculative)
    }
    if (!__any(pl != kPairEmpty)) break;
    if (pl != kPairEmpty) {
      if (leaf(pl)) { e = kPairEmpty; sp = 1; }  // shadowed: done
      pl = kPairEmpty;
    }
  }
}

// Block-wide copy of n 16-B chunks from global memory into LDS with eight
// loads in flight per thread (one load-wait-store per chunk left the staging
// latency-bound: ~9K cycles per block for the C3 scene). Every thread of the
// block calls it; the caller synchronises.
__device__ __forceinline__ void stage_lds(uint4* dst, const uint4* src, int n) {
  const int bd = (int)blockDim.x;
  int i = (int)threadIdx.x;
  for (; i + 7 * bd < n; i += 8 * bd) {
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = src[i + k * bd];
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[i + k * bd] = v[k];
  }
  for (; i < n; i += bd) dst[i] = src[i];
}

// Per-lane traversal of the hierarchy over the other bounded records
// (general-transform spheres, cubes, cylinders with finite caps; global
// memory, private stack): the same culling rule and exactness argument as the
// sphere hierarchy (DESIGN.md "Exact culling"). Scenes made of diagonal
// spheres and planes (C3, C5) have no such hierarchy.
template <bool SHADOW>
__device__ __forceinline__ void other_trace(const DevScene& sc, V3 o, V3 d, double t_shadow, Hit& h,
                                            unsigned& n_disc, unsigned& n_tests, unsigned& n_boxes) {
  if (sc.n_obvh == 0 || (SHADOW && h.key >= 0 && h.t < t_shadow)) return;
  const BvhNode* nodes = sc.obvh;
  float M[3];
  for (int ax = 0; ax < 3; ++ax)  // the root's two child boxes contain every box below them
    M[ax] = fmaxf(fmaxf(fabsf(nodes[0].lo[0][ax]), fabsf(nodes[0].hi[0][ax])),
                  fmaxf(fabsf(nodes[0].lo[1][ax]), fabsf(nodes[0].hi[1][ax])));
  const SlabRay sr = slab_ray(o, d, M);
  float t_hi = f32_up(SHADOW ? t_shadow : h.t);
  int stk[kBvhMaxDepth + 4];
  int sp = 0, e = 0;
  while (e != kBvhEmpty) {
    if (e >= 0) {
      const BvhNode& nd = nodes[e];
      float t0 = 0.0f, t1 = 0.0f;
      const bool h0 = slab_hit32(nd.lo[0], nd.hi[0], sr, t_hi, t0);
      const bool h1 = nd.child[1] != kBvhEmpty && slab_hit32(nd.lo[1], nd.hi[1], sr, t_hi, t1);
      n_boxes += 2;
      if (h0 && h1) {
        const bool flip = t1 < t0;
        stk[sp++] = flip ? nd.child[0] : nd.child[1];
        e = flip ? nd.child[1] : nd.child[0];
      } else {
        e = h0 ? nd.child[0] : h1 ? nd.child[1] : (sp > 0 ? stk[--sp] : kBvhEmpty);
      }
    } else {
      const int code = -(e + 1), first = code >> 7, cnt = code & 127;
      for (int k = first; k < first + cnt; ++k) other_test<SHADOW>(sc, sc.orec + k, o, d, h, n_disc);
      n_tests += (unsigned)cnt;
      if constexpr (SHADOW) {
        if (h.key >= 0 && h.t < t_shadow) return;  // shadowed: done
      } else {
        t_hi = f32_up(h.t);
      }
      e = sp > 0 ? stk[--sp] : kBvhEmpty;
    }
  }
}

// The line hierarchy (rt_layout.hpp ConeCluster; DESIGN.md §5.2 "Open tubes
// and cones"): open tubes and cones with finite bounds, leaves of one record
// (more only where the builder cannot split). First cone_prepass: per cluster
// one test rules out that every member takes the reference's a ~ 0 branch
// (cone.rs:102-110) for this ray; the members of an open cluster are checked
// with the reference's own a (quad_test's operations) and those below EPSILON
// are tested in full. Then line_trace: a child is entered when its box meets
// the ray's line within [t_lo, t_hi] (radiance rays t_lo = -inf: every root at
// t <= t_hi, the containers' t < 0 ones included; shadow rays t_lo = 0, only
// [0, distance) blocks); a leaf's records are tested, but for the cones the
// pre-pass took (a cone whose a ~ 0 for this ray is skipped only when its
// cluster was open, i.e. when the pre-pass tested it; a cone whose cluster the
// bound ruled out is tested in full here, so a rounding slip in the bound would
// cost a test, never a root). Order-independent minima, so the visiting order
// is free.
__device__ __forceinline__ bool cone_cluster_open(cConeCluster g, V3 d) {
  const double dm = fmax(fmax(fabs(d.x), fabs(d.y)), fabs(d.z)), dm2 = dm * dm;
  const double v = g->q[0] * d.x * d.x + g->q[1] * d.y * d.y + g->q[2] * d.z * d.z +
                   2.0 * (g->q[3] * d.x * d.y + g->q[4] * d.x * d.z + g->q[5] * d.y * d.z);
  const double av = fabs(v), rr = g->r * dm2;
  // closed: |v| - r dm^2 >= EPSILON with a margin for this arithmetic (NaN: open)
  return !(av - rr - 0x1p-40 * (av + rr) >= kEpsilon);
}
// the reference's |a| < EPSILON test of a cone (quad_test's object direction, quad_local_intersect's a)
template <typename QP>
__device__ __forceinline__ bool cone_degenerate(QP q, V3 d) {
  const V3 ld = v3(q->m[0] * d.x + q->m[1] * d.y + q->m[2] * d.z, q->m[4] * d.x + q->m[5] * d.y + q->m[6] * d.z,
                   q->m[8] * d.x + q->m[9] * d.y + q->m[10] * d.z);
  const double a = ld.x * ld.x - ld.y * ld.y + ld.z * ld.z;
  return fabs(a) < kEpsilon;
}
template <bool SHADOW>
__device__ __forceinline__ void cone_prepass(const DevScene& sc, V3 o, V3 d, Hit& h, unsigned& n_tests) {
  const cConeCluster cl = (cConeCluster)sc.lclus;
  const cQuadRec lrec = (cQuadRec)sc.lrec;
  for (int c = 0; c < sc.n_lclus; ++c) {  // wave-uniform: the clusters and their members in scalar loads
    if (!cone_cluster_open(cl + c, d)) continue;
    const int first = cl[c].first, count = cl[c].count;
    for (int j = first; j < first + count; ++j) {
      const cQuadRec q = lrec + ((const RT_CONST int32_t*)sc.lcone)[j];
      if (!cone_degenerate(q, d)) continue;
      quad_test<SHADOW>(q, o, d, h);
      ++n_tests;
    }
  }
}
template <bool SHADOW>
__device__ __forceinline__ void line_trace(const DevScene& sc, V3 o, V3 d, double t_shadow, Hit& h,
                                           unsigned& n_tests, unsigned& n_boxes) {
  if (sc.n_lbvh == 0) return;
  cone_prepass<SHADOW>(sc, o, d, h, n_tests);
  if (SHADOW && h.key >= 0 && h.t < t_shadow) return;
  const BvhNode* nodes = sc.lbvh;
  float M[3];
  for (int ax = 0; ax < 3; ++ax)  // the root's two child boxes contain every box below them
    M[ax] = fmaxf(fmaxf(fabsf(nodes[0].lo[0][ax]), fabsf(nodes[0].hi[0][ax])),
                  fmaxf(fabsf(nodes[0].lo[1][ax]), fabsf(nodes[0].hi[1][ax])));
  const SlabRay sr = slab_ray(o, d, M);
  const float t_lo = SHADOW ? 0.0f : -INFINITY;
  float t_hi = f32_up(SHADOW ? t_shadow : h.t);
  auto box = [&](const float* lo, const float* hi) {  // slab_hit32's test over [t_lo, t_hi]
    const float x0 = fmaf(lo[0], sr.inv[0], -sr.c_lo[0]), x1 = fmaf(hi[0], sr.inv[0], -sr.c_hi[0]);
    const float y0 = fmaf(lo[1], sr.inv[1], -sr.c_lo[1]), y1 = fmaf(hi[1], sr.inv[1], -sr.c_hi[1]);
    const float z0 = fmaf(lo[2], sr.inv[2], -sr.c_lo[2]), z1 = fmaf(hi[2], sr.inv[2], -sr.c_hi[2]);
    const float tmin = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), t_lo));
    const float tmax = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t_hi));
    return tmin <= tmax;
  };
  int stk[kBvhMaxDepth + 4];
  int sp = 0, e = 0;
  while (e != kBvhEmpty) {
    const BvhNode& nd = nodes[e];
    int next[2], nn = 0;
    for (int c = 0; c < 2; ++c) {
      const int32_t code = nd.child[c];
      if (code == kBvhEmpty) continue;
      ++n_boxes;
      if (!box(nd.lo[c], nd.hi[c])) continue;
      if (code >= 0) { next[nn++] = code; continue; }
      const int lc = -(code + 1), first = lc >> 7, cnt = lc & 127;
      for (int k = first; k < first + cnt; ++k) {
        const QuadRec* q = sc.lrec + k;
        if (q->kind == 4 && cone_degenerate(q, d)) {
          const int32_t cc = sc.lrec_clus[k];
          if (cc >= 0 && cone_cluster_open((cConeCluster)sc.lclus + cc, d)) continue;  // the pre-pass tested it
        }
        quad_test<SHADOW>(q, o, d, h);
        ++n_tests;
        if constexpr (SHADOW) {
          if (h.key >= 0 && h.t < t_shadow) return;  // shadowed: done
        } else {
          t_hi = f32_up(h.t);
        }
      }
    }
    if (nn == 2) stk[sp++] = next[1];
    e = nn > 0 ? next[0] : (sp > 0 ? stk[--sp] : kBvhEmpty);
  }
}
// Counted launches (the reference's shape tests come from the group gates
// each ray met, GateSkips): the gates of the grouped records the other
// records' hierarchy holds (trace_rest counts those of the records it loops
// over; the line hierarchy holds no grouped record). Every record is visited
// here, so only counted launches call it.
__device__ __forceinline__ void count_hier_gates(const DevScene& sc, V3 o, V3 d, GateSkips& sk) {
  if (!sc.n_groups) return;
  const cQuadRec orec = (cQuadRec)sc.orec;
  for (int k = 0; k < sc.n_orec; ++k) {
    const int g = orec[k].gate;
    if (g && !group_gate(sc, g, o, d)) {
      if (orec[k].kind == 0) ++sk.sph; else ++sk.other;
    }
  }
}

__host__ __device__ inline size_t lane_stack_bytes(int depth) { return (size_t)(depth > 0 ? depth : 1) * kTraceBlock * 4; }
__host__ __device__ inline size_t sph_lds_bytes(const DevScene& sc) { return (size_t)sc.n_diag * sizeof(SphereDiag); }
// the pair image's sphere records: 48 B each, then the metas (Sph48)
__host__ __device__ inline size_t sph48_lds_bytes(const DevScene& sc) {
  return (size_t)sc.n_diag * 48 + (((size_t)sc.n_diag * 4 + 15) & ~(size_t)15);
}
// The light buffer's distances in LDS as binary16 lower bounds of the binary32
// ones (2 B each): a stored value never exceeds the true distance, so a walk
// that stops at the first stored distance beyond the origin stops no earlier
// than the exact walk would (lb_walk).
__host__ __device__ inline size_t delta_lds_bytes(const DevScene& sc) {
  return sc.lb_cells ? (((size_t)sc.n_lights * sc.n_diag * sizeof(_Float16) + 15) & ~(size_t)15) : 0;
}
// LANE 14: [16-bit stack (bvh_depth + 1 with the sentinel) x kTraceBlock][pair nodes][Sph48 records]
// (no pair image without the scene's 16-bit pair codes: rt_bvh.cpp pair_layout)
__host__ __device__ inline size_t pair_lds_bytes(const DevScene& sc) {
  if (!sc.bvh_pair) return (size_t)1 << 40;
  return ((lane_stack_bytes(sc.bvh_depth + 1) / 2 + 15) & ~(size_t)15) + (size_t)sc.n_bvh * sizeof(BvhNode) +
         sph48_lds_bytes(sc);
}
// LANE 4: the 16-bit stack (sc.bvhw_stack entries) x kTraceBlock, before the distances and the treelet
__host__ __device__ inline size_t wide_stack_bytes(const DevScene& sc) {
  return ((size_t)(sc.bvhw_stack > 0 ? sc.bvhw_stack : 1) * kTraceBlock * 2 + 15) & ~(size_t)15;
}
// LANE 15: [16-bit stack][every wide node][Sph48 records]
__host__ __device__ inline size_t wide_lds_bytes(const DevScene& sc) {
  if (!sc.bvhw) return (size_t)1 << 40;
  return wide_stack_bytes(sc) + (size_t)sc.n_bvhw * sizeof(BvhWide) + sph48_lds_bytes(sc);
}
constexpr unsigned kLdsSpheres = 1u, kLdsDeltas = 2u;  // lane_scene's lds_flags (LANE 0: records; all: distances)

struct LaneScene {
  const unsigned char* nodes;  // pair layout in LDS (14) or BvhNode[] in global memory
  const SphereDiag* sd;        // sphere records (LDS or global; not LANE 14)
  Sph48 s48;                   // LANE 14: the sphere records in LDS
  uint16_t* stack16;           // LANE 14: the per-lane 16-bit LDS stack
  const float* delta;          // light buffer: per-light box distances (global)
  const _Float16* delta16;     // ... their binary16 lower bounds in LDS (when staged), else null
  int* stack;                  // per-lane LDS stack (14, 3) or the wave's stack (0)
  float M[3];                  // bound on |box coordinate| per axis (slab_ray)
  const BvhNode* top;          // 3: the LDS copy of the first n_top nodes
  int n_top;
  const BvhWide* wtop;         // 15: the LDS copy of the wide nodes
  const BvhWide16* wtop16;     // 4: the LDS copy of the first n_top binary16 wide nodes
};
template <int LANE>
__device__ __forceinline__ LaneScene lane_scene(const DevScene& sc, unsigned lds_flags, unsigned n_top, int* static_stack,
                                                unsigned char* dyn) {
  LaneScene ls{(const unsigned char*)sc.bvh, sc.sph_diag, Sph48{nullptr, nullptr}, nullptr, sc.lb_delta, nullptr,
               static_stack, {0.f, 0.f, 0.f}, nullptr, 0, nullptr, nullptr};
  unsigned char* p = dyn;
  if constexpr (LANE == 15) {  // [16-bit stack][every wide node][Sph48 records and metas]
    ls.stack16 = (uint16_t*)dyn + threadIdx.x;
    p += wide_stack_bytes(sc);
    stage_lds((uint4*)p, (const uint4*)sc.bvhw, sc.n_bvhw * (int)(sizeof(BvhWide) / 16));
    ls.wtop = (const BvhWide*)p;
    ls.nodes = p;
    ls.n_top = sc.n_bvhw;
    p += (size_t)sc.n_bvhw * sizeof(BvhWide);
    uint4* r = (uint4*)p;
    const uint4* src = (const uint4*)sc.sph_diag;
    const int n3 = sc.n_diag * 3, bd = (int)blockDim.x;
    for (int i = (int)threadIdx.x; i < n3; i += bd) {
      const int k = i / 3;
      r[i] = src[4 * k + (i - 3 * k)];
    }
    int* mt = (int*)(p + (size_t)sc.n_diag * 48);
    for (int k = (int)threadIdx.x; k < sc.n_diag; k += bd) mt[k] = (int)sc.sph_diag[k].meta;
    ls.s48 = Sph48{(const double*)p, (const int*)mt};
    p += sph48_lds_bytes(sc);
  }
  if constexpr (LANE == 4) {  // [16-bit stack][distances][treelet of binary16 wide nodes]
    ls.stack16 = (uint16_t*)dyn + threadIdx.x;
    p += wide_stack_bytes(sc);
    ls.nodes = (const unsigned char*)sc.bvhw16;
    if (n_top > 0) {
      unsigned char* q = p + ((lds_flags & kLdsDeltas) ? delta_lds_bytes(sc) : 0);
      stage_lds((uint4*)q, (const uint4*)sc.bvhw16, (int)n_top * (int)(sizeof(BvhWide16) / 16));
      ls.wtop16 = (const BvhWide16*)q;
      ls.n_top = (int)n_top;
    }
  }
  if constexpr (LANE == 14) {
    // pair layout (BvhPair): per axis, the two children's lower bounds form one
    // 8-B pair and their upper bounds the next (lane_trace_pair)
    ls.stack16 = (uint16_t*)dyn + threadIdx.x;
    p += (lane_stack_bytes(sc.bvh_depth + 1) / 2 + 15) & ~(size_t)15;
    stage_lds((uint4*)p, (const uint4*)sc.bvh_pair, sc.n_bvh * (int)(sizeof(BvhPair) / 16));
    ls.nodes = p;
    p += (size_t)sc.n_bvh * sizeof(BvhPair);
    // the sphere records, 48 B each (three of a SphereDiag's four 16-B chunks), and the metas
    {
      uint4* r = (uint4*)p;
      const uint4* src = (const uint4*)sc.sph_diag;
      const int n3 = sc.n_diag * 3, bd = (int)blockDim.x;
      for (int i = (int)threadIdx.x; i < n3; i += bd) {
        const int k = i / 3;
        r[i] = src[4 * k + (i - 3 * k)];
      }
      int* mt = (int*)(p + (size_t)sc.n_diag * 48);
      for (int k = (int)threadIdx.x; k < sc.n_diag; k += bd) mt[k] = (int)sc.sph_diag[k].meta;
      ls.s48 = Sph48{(const double*)p, (const int*)mt};
      p += sph48_lds_bytes(sc);
    }
  }
  if (LANE == 0 && (lds_flags & kLdsSpheres)) {
    stage_lds((uint4*)p, (const uint4*)sc.sph_diag, sc.n_diag * (int)(sizeof(SphereDiag) / 16));
    ls.sd = (const SphereDiag*)p;
    p += sph_lds_bytes(sc);
  }
  if (LANE == 3 && n_top > 0) {  // the treelet: after the distances when those are staged
    unsigned char* q = p + ((lds_flags & kLdsDeltas) ? delta_lds_bytes(sc) : 0);
    stage_lds((uint4*)q, (const uint4*)sc.bvh, (int)n_top * (int)(sizeof(BvhNode) / 16));
    ls.top = (const BvhNode*)q;
    ls.n_top = (int)n_top;
  }
  if (lds_flags & kLdsDeltas) {
    // binary16 lower bounds: a positive value rounded toward zero (= down), anything
    // else 0 (a stored 0 never ends a walk: the walk compares with a positive distance)
    _Float16* ld = (_Float16*)p;
    auto down16 = [](float v) -> _Float16 { return v > 0.0f ? __builtin_amdgcn_cvt_pkrtz(v, 0.0f)[0] : (_Float16)0.0f; };
    const int nd = sc.n_lights * sc.n_diag, bd = (int)blockDim.x;
    int i = (int)threadIdx.x;
    for (; i + 7 * bd < nd; i += 8 * bd) {  // eight loads in flight per thread
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = sc.lb_delta[i + k * bd];
#pragma unroll
      for (int k = 0; k < 8; ++k) ld[i + k * bd] = down16(v[k]);
    }
    for (; i < nd; i += bd) ld[i] = down16(sc.lb_delta[i]);
    ls.delta16 = ld;
  }
  __syncthreads();
  for (int ax = 0; ax < 3; ++ax) {  // the root's two child boxes contain every box below them
    float m = 0.0f;
    if (sc.n_bvh > 0) {
      const BvhNode& r = sc.bvh[0];
      m = fmaxf(fmaxf(fabsf(r.lo[0][ax]), fabsf(r.hi[0][ax])), fmaxf(fabsf(r.lo[1][ax]), fabsf(r.hi[1][ax])));
    }
    ls.M[ax] = m;
  }
  return ls;
}

// World::is_shadowed for the diagonal spheres through the light buffer
// (DESIGN.md "Light buffer"): the cube-map cell of direction o - light lists
// every sphere that can block the ray, nearest box first; the walk stops at
// the first blocker or at the first box farther from the light than the
// origin. One 16-B load brings the cell's first kLbInline entries. An origin
// beyond the light's validity radius (or non-finite) tests every sphere.
template <typename SD>  // the sphere records: const SphereDiag* (global or LDS) or Sph48 (the pair image)
__device__ __forceinline__ void lb_walk(const DevScene& sc, SD sd, const float* delta, const _Float16* delta16,
                                        unsigned l, V3 o, V3 d, double dist, Hit& h, unsigned& n_disc,
                                        unsigned& n_tests, int skip = -1) {
  cLightRec Lr = (cLightRec)sc.lights + l;
  if (dist <= (double)sc.lb_limit[l] && dist >= 1e-30) {
    const int R = sc.lb_res;
    const unsigned per_light = 6u * (unsigned)R * (unsigned)R;
    const float half_r = 0.5f * (float)R;
    // w = o - light (= -(light - o) bit for bit), in binary32
    const float wx = (float)(o.x - Lr->pos[0]), wy = (float)(o.y - Lr->pos[1]), wz = (float)(o.z - Lr->pos[2]);
    const float ax = fabsf(wx), ay = fabsf(wy), az = fabsf(wz);
    unsigned f;
    float wa, wb, wc;
    if (ax >= ay && ax >= az) { f = wx < 0.0f ? 1u : 0u; wa = ax; wb = wy; wc = wz; }
    else if (ay >= az) { f = wy < 0.0f ? 3u : 2u; wa = ay; wb = wz; wc = wx; }
    else { f = wz < 0.0f ? 5u : 4u; wa = az; wb = wx; wc = wy; }
    // (an approximate reciprocal: within 2 ulp, 2.4e-7 of the cube-face coordinate, far inside the
    // host's 1e-5 margins)
    const float rwa = __builtin_amdgcn_rcpf(wa);
    const float u = fminf(fmaxf(wb * rwa, -1.0f), 1.0f), v = fminf(fmaxf(wc * rwa, -1.0f), 1.0f);
    const unsigned iu = (unsigned)min((int)((u + 1.0f) * half_r), R - 1);
    const unsigned iv = (unsigned)min((int)((v + 1.0f) * half_r), R - 1);
    const LbCell c = sc.lb_cells[l * per_light + (f * (unsigned)R + iv) * (unsigned)R + iu];
    const unsigned cnt = c.w0 & 0xFFFFu;
    // the inline entries as a queue of 16-bit indices: idx0..idx3 in q, idx4 in c.w2 >> 16
    unsigned long long q = (unsigned long long)(c.w0 >> 16) | (unsigned long long)c.w1 << 16 |
                           (unsigned long long)(c.w2 & 0xFFFFu) << 48;
    const float* dl = delta + (size_t)l * sc.n_diag;
    const _Float16* dl16 = delta16 ? delta16 + (size_t)l * sc.n_diag : nullptr;
    const float dist_up = f32_up(dist);
    for (unsigned k = 0; k < cnt; ++k) {
      unsigned idx;
      if (k < 4u) { idx = (unsigned)(q & 0xFFFFu); q >>= 16; }
      else if (k == 4u) idx = c.w2 >> 16;
      else idx = sc.lb_ov[c.ov + k - (unsigned)kLbInline];
      if ((dl16 ? (float)dl16[idx] : dl[idx]) > dist_up) break;  // this box and all after it lie beyond the origin
      if ((int)idx == skip) continue;
      leaf_sphere_test<true>(sd, (int)idx, o, d, h, n_disc);
      ++n_tests;
      if (h.key >= 0 && h.t < dist) break;
    }
  } else {
    for (int k = 0; k < sc.n_diag; ++k) {
      if (k == skip) continue;
      leaf_sphere_test<true>(sd, k, o, d, h, n_disc);
      ++n_tests;
      if (h.key >= 0 && h.t < dist) break;
    }
  }
}

// World::is_shadowed (world.rs:95-105) of the ray from `o` towards light `l`
// (direction d, distance dist): the records outside the BVH first (any hit
// before the light ends the ray), then the light buffer, or the BVH of the
// kernel's image when the scene has no light buffer.
// `first` >= 0: a sphere record tested before everything else (shade_fused: the
// sphere whose inside the point lies on). is_shadowed asks whether ANY
// shadow-casting object meets the ray before the light, so a blocker found
// first is the answer whatever the others hold; the ray leaves that sphere
// through its far side, before a light outside it.
// `skip` >= 0: a sphere record the light-buffer walk leaves out (shade_fused:
// the sphere hit from outside, the light in front of the surface, i.e. the
// computed light . normal >= 0, and the record flagged kOwnOutside). Every
// point o + t d (t >= 0) then lies at least ~EPSILON beyond the tangent plane
// at the hit (the over point's step; the computed direction's error moves the
// ray by 1e-16 t), outside the convex ellipsoid; in object space the ray keeps
// at least EPSILON / r_max >= 1e-8 from the unit sphere, so the test's
// discriminant is negative or both roots negative, at margins eight orders
// above its rounding: the reference's test of that sphere never reports a
// blocker, and leaving it out changes no answer.
template <int LANE, bool QUADS>
__device__ __forceinline__ bool shadow_trace(const DevScene& sc, unsigned use_lb, const LaneScene& ls, unsigned l,
                                             V3 o, V3 d, double dist, unsigned& n_disc, unsigned& n_tests,
                                             unsigned& n_boxes, GateSkips* skips = nullptr, int first = -1,
                                             int skip = -1) {
  Hit h;
  hit_init(h);
  if (first >= 0) {
    if constexpr (LANE == 14 || LANE == 15) leaf_sphere_test<true>(ls.s48, first, o, d, h, n_disc);
    else leaf_sphere_test<true>(ls.sd, first, o, d, h, n_disc);
    ++n_tests;
    if (h.key >= 0 && h.t < dist) return true;
  }
  trace_rest<true, QUADS, true>(sc, o, d, h, n_disc, skips);
  if constexpr (QUADS) {
    other_trace<true>(sc, o, d, dist, h, n_disc, n_tests, n_boxes);
    line_trace<true>(sc, o, d, dist, h, n_tests, n_boxes);
  }
  if (!(h.key >= 0 && h.t < dist)) {
    if (use_lb) {
      if constexpr (LANE == 14 || LANE == 15) lb_walk(sc, ls.s48, ls.delta, ls.delta16, l, o, d, dist, h, n_disc, n_tests, skip);
      else lb_walk(sc, ls.sd, ls.delta, ls.delta16, l, o, d, dist, h, n_disc, n_tests, skip);
    } else if constexpr (LANE == 14) {
      lane_trace_pair<true>(ls.nodes, ls.s48, ls.M, sc.n_bvh > 0, o, d, dist, h, n_disc, n_tests, n_boxes,
                            ls.stack16);
    } else if constexpr (LANE == 15) {
      lane_trace_wide<true, Sph48, true>((const BvhWide*)ls.nodes, ls.s48, ls.M, sc.bvhw != nullptr, o, d, dist, h, n_disc,
                                         n_tests, n_boxes, ls.stack16, ls.wtop, ls.n_top, sc.n_diag);
    } else if constexpr (LANE == 4) {
      lane_trace_wide<true>((const BvhWide16*)ls.nodes, ls.sd, ls.M, sc.bvhw16 != nullptr, o, d, dist, h, n_disc,
                            n_tests, n_boxes, ls.stack16, ls.wtop16, ls.n_top, sc.n_diag);

    } else if constexpr (LANE == 0) {
      Hit hb;  // the wave traversal starts from an empty hit; any blocker is an answer
      bvh_trace<false, true>(sc, nullptr, ls.stack, o, d, dist, hb, n_disc, n_tests, n_boxes);
      if (hb.key >= 0 && hb.key != 0x7fffffff && hb.t < dist) h = hb;
    } else {
      lane_trace<true, LANE == 3>((const BvhNode*)ls.nodes, ls.sd, ls.M, sc.n_bvh > 0, o, d, dist, h, n_disc,
                                  n_tests, n_boxes, ls.stack, ls.top, ls.n_top);
    }
  }
  hit_finish(h);
  return h.key >= 0 && h.t < dist;
}

// World::shade_hit's combination (world.rs:58-67) of the surface term and the
// reflected / refracted colours, with the reference's expression.
// (From the material's reflective and transparency values alone: wf_combine_parents
// reads them from the scene's small per-object table.)
__device__ __forceinline__ V3 shade_color_rt(double reflective, double transparency, V3 surface, V3 refl, V3 refr,
                                             double schlick_r) {
  if (reflective > 0.0 && transparency > 0.0)
    return vadd(vadd(surface, vscale(refl, schlick_r)), vscale(refr, 1.0 - schlick_r));
  return vadd(vadd(surface, refl), refr);
}
__device__ __forceinline__ V3 shade_color(const ShadeRec& m, V3 surface, V3 refl, V3 refr, double schlick_r) {
  return shade_color_rt(m.reflective, m.transparency, surface, refl, refr, schlick_r);
}


typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
// Streaming loads and stores of the fused kernels: rays, parents and colours
// are written once and read once by a later launch, so they are marked
// non-temporal and leave the L2 to the scene (C3 0.947 -> 0.929 ms, C5 60.0
// -> 58.8 ms per frame). The same marking in wf_combine_parents cost 2 %.
__device__ __forceinline__ void st_d(double* p, double v) { __builtin_nontemporal_store(v, p); }

}  // namespace rtamd
