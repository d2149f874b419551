// rt_persist.hip — the persistent frame kernel (rt_persist.hpp): ONE launch
// per frame, all recursion depths, shade_hit's combine folded in.
//
// This file is compiled twice (Makefile): with -DRT_PS_LDS_IMAGE for the
// scene image in LDS (pair-layout nodes, sphere records and per-lane stacks:
// the C3 headline), and without it for scenes whose image does not fit
// (nodes and records in global memory with an LDS stack and treelet, or a
// scratch stack: C5). The two objects get their own code generation flags.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "rt_device.hpp"
#include "rt_persist.hpp"
#include "rt_trace.hpp"
#include "rt_wavefront.hpp"

#pragma clang fp contract(off)

namespace rtamd {

enum : unsigned { PS_EXIT = 0u, PS_ROOTS = 1u, PS_QUEUED = 2u };
// a wait (for work another wave is producing, or for an earlier append to be
// published) longer than this many 100-MHz ticks (2 s) abandons the frame and
// raises the workspace's fault flag instead of hanging the device
constexpr unsigned long long kPsWaitTicks = 200000000ull;

// Scheduler state of a workgroup (LDS). Ring entries [head, commit) are
// published and unclaimed, [commit, tail) reserved by waves still writing.
struct PsSched {
  unsigned head, tail, commit, busy;
  unsigned roots_done;  // no camera chunk is left for this workgroup
  unsigned tree_free;   // bit t: tree slot t holds no rays
  unsigned cls_done;    // bit c: chunk class c is exhausted
  unsigned pad;
  int live[kPsMaxTrees];         // rays of tree t not yet finished (queued, being traced, or published)
  unsigned root0[kPsMaxTrees];   // root index of tree t's first ray (its camera chunk * 64)
  unsigned lvl[kPsMaxTrees][kPsMaxDepth];  // nodes with children of tree t per depth (its level lists)
};
static_assert(sizeof(PsSched) <= kPsSchedBytes, "PsSched exceeds its LDS budget (rt_persist.hpp)");

__device__ __forceinline__ unsigned ps_ld(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// every vector-memory access of this wave has completed (its stores are in
// the L2, where the workgroup's other waves read them)
__device__ __forceinline__ void ps_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

typedef double ps_d2 __attribute__((ext_vector_type(2)));
typedef unsigned ps_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ps_st2(void* p, double x, double y) {
  __builtin_nontemporal_store((ps_d2){x, y}, (ps_d2*)p);
}
__device__ __forceinline__ ps_d2 ps_ld2(const void* p) { return __builtin_nontemporal_load((const ps_d2*)p); }

// A wait exceeded its time bound: record what this wave saw (host-mapped,
// read back in the library's error text), then the code (word 0).
// (Everything by value: a reference to the kernel's arguments would put them in scratch.)
__device__ __noinline__ void ps_fault(int* fault, unsigned trees, unsigned q_cap, const PsSched& S, int code,
                                      unsigned it, unsigned long long dt) {
  volatile int* f = fault;
  f[1] = (int)blockIdx.x; f[2] = (int)(threadIdx.x >> 6);
  f[3] = (int)S.head; f[4] = (int)S.tail; f[5] = (int)S.commit; f[6] = (int)S.busy;
  f[7] = (int)S.roots_done; f[8] = (int)S.tree_free; f[9] = (int)S.cls_done;
  f[10] = (int)it; f[11] = (int)(dt & 0xFFFFFFFFull); f[12] = (int)(dt >> 32);
  for (int k = 0; k < 8; ++k) f[13 + k] = S.live[k];
  f[21] = (int)gridDim.x; f[22] = (int)trees; f[23] = (int)q_cap;
  f[0] = code;
}

// The next camera chunk for this workgroup: class counters first its own
// (blocks are dealt round-robin to the XCDs), then the others'.
__device__ __forceinline__ unsigned ps_next_chunk(PsSched& S, const PsArgs& a, unsigned n_chunks) {
  const unsigned X = gridDim.x < kPsClasses ? gridDim.x : kPsClasses;
  const unsigned c0 = blockIdx.x % X;
  for (unsigned k = 0; k < X; ++k) {
    const unsigned cls = c0 + k < X ? c0 + k : c0 + k - X;
    if (ps_ld(&S.cls_done) >> cls & 1u) continue;
    const unsigned j = atomicAdd(&a.ctr->chunk[cls * kPsCtrStride], 1u);
    const unsigned ch = cls + X * j;
    if (ch < n_chunks) return ch;
    atomicOr(&S.cls_done, 1u << cls);
  }
  return ~0u;
}

// Work for one wave (run by its lane 0): a full chunk of queued rays, else a
// new camera chunk (when a tree slot is free), else the queued rays there
// are, else wait while another wave may still publish rays; PS_EXIT once the
// workgroup's camera chunks are gone and nothing is queued or being traced.
__device__ void ps_acquire(PsSched& S, const PsArgs& a, unsigned n_chunks, unsigned& kind, unsigned& base,
                           unsigned& take, unsigned& tree) {
  unsigned long long t0 = 0;
  unsigned waits = 0;
  for (unsigned it = 0;; ++it) {
    atomicAdd(&S.busy, 1u);
    unsigned h = ps_ld(&S.head), c = ps_ld(&S.commit);
    if (c - h >= 64u) {
      if (atomicCAS(&S.head, h, h + 64u) == h) {
        kind = PS_QUEUED; base = h; take = 64u;
        return;
      }
      atomicSub(&S.busy, 1u);
      continue;
    }
    if (!ps_ld(&S.roots_done)) {
      unsigned m = ps_ld(&S.tree_free);
      int got = -1;
      while (m) {
        const unsigned b = (unsigned)__ffs(m) - 1u;
        const unsigned old = atomicAnd(&S.tree_free, ~(1u << b));
        if (old >> b & 1u) { got = (int)b; break; }
        m = old & ~(1u << b);
      }
      if (got >= 0) {
        const unsigned ch = ps_next_chunk(S, a, n_chunks);
        if (ch != ~0u) {
          const unsigned n = min(64u, a.n0 - ch * 64u);
          S.live[got] = (int)n;
          S.root0[got] = ch * 64u;
          kind = PS_ROOTS; base = ch; take = n; tree = (unsigned)got;
          return;
        }
        atomicOr(&S.tree_free, 1u << got);
        atomicOr(&S.roots_done, 1u);
      }
    }
    h = ps_ld(&S.head);
    c = ps_ld(&S.commit);
    // policy 1: fewer than 64 queued rays only when no other wave can add to them
    if (c != h && (a.policy == 0u || ps_ld(&S.roots_done) || ps_ld(&S.busy) <= 1u)) {
      const unsigned n = min(64u, c - h);
      if (atomicCAS(&S.head, h, h + n) == h) {
        kind = PS_QUEUED; base = h; take = n;
        return;
      }
      atomicSub(&S.busy, 1u);
      continue;
    }
    const unsigned busy = atomicSub(&S.busy, 1u) - 1u;
    if (busy == 0u && ps_ld(&S.roots_done) && ps_ld(&S.head) == ps_ld(&S.tail)) {
      kind = PS_EXIT;
      return;
    }
    if ((waits++ & 63u) == 0u) {  // the clock starts at this wave's first wait (not at a lost CAS)
      const unsigned long long now = __builtin_amdgcn_s_memrealtime();
      if (waits == 1u) {
        t0 = now;
      } else if (now - t0 > kPsWaitTicks) {
        ps_fault(a.fault, a.trees, a.q_cap, S, 2, it, now - t0);
        kind = PS_EXIT;
        return;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Root ray i of the render: sample `smp` of a pixel of the shard
// (camera.rs:57-69 / 71-90), or ray i of a color_at batch.
__device__ __forceinline__ void ps_root_ray(const PsArgs& a, const DevCamera& cam, unsigned i, V3& o, V3& d) {
  if (a.camera_mode) {
    uint32_t x, lr, smp;
    gen0_pixel(a.aa, a.rows, cam.hsize, i, x, lr, smp);
    const uint32_t blk = lr / a.row_block, off = lr - blk * a.row_block;
    const uint32_t y = (blk * a.n_shards + a.shard) * a.row_block + off;
    if (a.aa == 1) {
      ray_for_pixel(cam, x, y, o, d);
    } else {
      const double* ofs = kAaOffsets[a.aa - 1 + smp];
      ray_for_pixel(cam, x, y, o, d, ofs[0], ofs[1]);
    }
  } else {
    const double* r = a.in_rays + (size_t)i * 6;
    o = v3(r[0], r[1], r[2]);
    d = v3(r[3], r[4], r[5]);
  }
}
// Where root ray i's colour goes: the canvas (camera, aa == 1: ray order is
// tile order, the canvas row-major) or slot i (AA samples, batches).
__device__ __forceinline__ double* ps_root_dst(const PsArgs& a, const DevCamera& cam, unsigned i) {
  size_t oi = i;
  if (a.camera_mode && a.aa == 1) {
    uint32_t x, lr, smp;
    gen0_pixel(1u, a.rows, cam.hsize, i, x, lr, smp);
    oi = (size_t)lr * cam.hsize + x;
  }
  return a.out + oi * 3;
}

// Tree t is finished (every ray of its 64 roots has been traced and every
// node without children has written its colour into its parent's record):
// evaluate shade_hit's combination (world.rs:58-67; the reflected colour is
// color_at(reflect ray) * reflective, world.rs:113, the refracted one
// * transparency, world.rs:133) for its nodes with children, deepest level
// first, one node per lane; a level's colours go into the next level's
// records (or, at the roots, the output) before that level is read.
// Run by one whole wave.
__device__ __forceinline__ void ps_combine_tree(const DevScene& sc, const PsArgs& a, const DevCamera& cam,
                                                PsParent* par, const uint16_t* lists, PsSched& S, unsigned t) {
  const unsigned lane = lane_id();
  for (int g = (int)a.max_depth - 1; g >= 0; --g) {
    const unsigned cnt = S.lvl[t][g];
    const uint16_t* lst = lists + ((size_t)t * (64u * a.n_int) + 64u * ((1u << g) - 1u));
    for (unsigned i = lane; i < cnt; i += 64u) {
      const unsigned e = __builtin_nontemporal_load(lst + i);
      const unsigned px = e >> 10, node = e & 1023u;
      const PsParent* P = par + ((size_t)t * 64u + px) * a.n_int + node;
      const ps_d2 s01 = ps_ld2(P->surface), s2k = ps_ld2(&P->surface[2]);
      const ps_u4 tl = __builtin_nontemporal_load((const ps_u4*)&P->obj);
      const ShadeRec& m = sc.shade[(int)tl.x];
      V3 refl = v3(0.0, 0.0, 0.0), refr = v3(0.0, 0.0, 0.0);
      if (tl.y & 1u) {
        const ps_d2 q = ps_ld2(P->refl);
        refl = vscale(v3(q.x, q.y, __builtin_nontemporal_load(&P->refl[2])), m.reflective);
      }
      if (tl.y & 2u) {
        const ps_d2 q = ps_ld2(P->refr);
        refr = vscale(v3(q.x, q.y, __builtin_nontemporal_load(&P->refr[2])), m.transparency);
      }
      const V3 col = shade_color(m, v3(s01.x, s01.y, s2k.x), refl, refr, s2k.y);
      double* dst;
      if (node == 0u) {
        dst = ps_root_dst(a, cam, S.root0[t] + px);
      } else {
        PsParent* Q = par + ((size_t)t * 64u + px) * a.n_int + ((node - 1u) >> 1);
        dst = ((node - 1u) & 1u) ? Q->refr : Q->refl;
      }
      ps_st2(dst, col.x, col.y);
      __builtin_nontemporal_store(col.z, dst + 2);
    }
    ps_drain();  // this level's colours are in the L2 before the next level reads them
  }
  if (lane < kPsMaxDepth) S.lvl[t][lane] = 0u;
}

struct PsTally {
  unsigned disc = 0, tests = 0, boxes = 0;
  unsigned sh_disc = 0, sh_tests = 0, sh_boxes = 0, sh_rays = 0;
};
// shader clock (counted launches only: where a wave's time goes)
template <bool TALLY>
__device__ __forceinline__ unsigned long long ps_clock() {
  if constexpr (TALLY) return __builtin_amdgcn_s_memtime();
  return 0ull;
}

// One frame. LANE: the scene image (rt_trace.hpp lane_scene: 14 = pair
// layout in LDS, 3 = global nodes with an LDS stack and treelet, 1 = global
// nodes, scratch stack). TALLY: a counted launch (work tallies for stats).
template <int LANE, bool QUADS, bool TALLY>
__global__ __launch_bounds__(kTraceBlock, 4) void ps_render(DevScene sc, DevCamera cam, PsArgs a) {
  __shared__ int stack_lds[LANE == 3 ? kLaneLdsDepth * kTraceBlock : 1];
  __shared__ PsSched S;
  extern __shared__ __attribute__((aligned(16))) unsigned char lane_dyn[];
  if (threadIdx.x == 0) {
    S.head = 0u; S.tail = 0u; S.commit = 0u; S.busy = 0u;
    S.roots_done = 0u; S.cls_done = 0u;
    S.tree_free = a.trees >= 32u ? 0xFFFFFFFFu : (1u << a.trees) - 1u;
  }
  for (unsigned k = threadIdx.x; k < kPsMaxTrees * kPsMaxDepth; k += blockDim.x) (&S.lvl[0][0])[k] = 0u;
  const LaneScene ls = lane_scene<LANE>(sc, a.lds_flags, a.n_top, stack_lds + threadIdx.x, lane_dyn);
  const unsigned lane = lane_id();
  const unsigned n_chunks = (a.n0 + 63u) / 64u;
  const unsigned L = (unsigned)sc.n_lights;
  PsRay* ring = a.rings + (size_t)blockIdx.x * a.q_cap;
  PsParent* par = a.parents + (size_t)blockIdx.x * a.trees * 64u * a.n_int;
  uint16_t* lists = a.lists + (size_t)blockIdx.x * a.trees * 64u * a.n_int;
  WfCounters* cnt = (WfCounters*)a.cnt;
  PsTally tl;
  for (;;) {
    unsigned kind = 0, base = 0, take = 0, tree = 0;
    const unsigned long long c0 = ps_clock<TALLY>();
    if (lane == 0) ps_acquire(S, a, n_chunks, kind, base, take, tree);
    kind = (unsigned)__builtin_amdgcn_readfirstlane((int)kind);  // lane 0's answer, wave-uniform
    if (kind == PS_EXIT) break;
    const unsigned long long c1 = ps_clock<TALLY>();
    base = (unsigned)__builtin_amdgcn_readfirstlane((int)base);  // lane 0's answer, wave-uniform
    take = (unsigned)__builtin_amdgcn_readfirstlane((int)take);  // lane 0's answer, wave-uniform
    tree = (unsigned)__builtin_amdgcn_readfirstlane((int)tree);  // lane 0's answer, wave-uniform
    // ---- this lane's ray: a camera (or batch) root, or a queued child
    const bool valid = lane < take;
    unsigned t = tree, px = lane, node = 0;
    V3 o = v3(0.0, 0.0, 0.0), d = v3(0.0, 0.0, 0.0);
    if (valid) {
      if (kind == PS_ROOTS) {
        ps_root_ray(a, cam, base * 64u + lane, o, d);
      } else {
        const PsRay* r = ring + (base + lane) % a.q_cap;
        const ps_d2 q0 = ps_ld2(&r->o[0]), q1 = ps_ld2(&r->o[2]), q2 = ps_ld2(&r->d[1]);
        const unsigned id = __builtin_nontemporal_load(&r->id);
        o = v3(q0.x, q0.y, q1.x);
        d = v3(q1.y, q2.x, q2.y);
        t = id >> 16;
        px = (id >> 10) & 63u;
        node = id & 1023u;
      }
    }
    // ---- World::intersect + hit (world.rs:31-38, intersection.rs:108-120)
    Hit h;
    hit_init(h);
    if (valid) {
      // planes and the other records first: an early nearest hit tightens the culling
      trace_rest<false, QUADS, true>(sc, o, d, h, tl.disc);
      if constexpr (QUADS) other_trace<false>(sc, o, d, 0.0, h, tl.disc, tl.tests, tl.boxes);
      if constexpr (LANE == 14)
        lane_trace_pair<false>(ls.nodes, ls.sd, ls.M, sc.n_bvh > 0, o, d, 0.0, h, tl.disc, tl.tests, tl.boxes,
                               ls.stack);
      else
        lane_trace<false, LANE == 3>((const BvhNode*)ls.nodes, ls.sd, ls.M, sc.n_bvh > 0, o, d, 0.0, h, tl.disc,
                                     tl.tests, tl.boxes, ls.stack, ls.top, ls.n_top);
    }
    hit_finish(h);
    const unsigned long long c2 = ps_clock<TALLY>();
    // ---- color_at's shading (world.rs:70-81, 40-68): prepare_computations,
    // the children, every light's shadow ray and lighting(). Only what the
    // lights loop and the spawn need stays live across the shadow traces; the
    // under point, reflect vector and refracted direction are formed after it
    // from the same operands with the same operations (the same bits).
    const unsigned g = 31u - (unsigned)__clz((int)(node + 1u));  // depth of heap node `node`
    const unsigned remaining = a.max_depth - g;
    bool hit = false, want_refl = false, want_refr = false;
    V3 point = v3(0.0, 0.0, 0.0), normal = v3(0.0, 0.0, 0.0), over = v3(0.0, 0.0, 0.0);
    double n_ratio = 0.0, k_refr = 0.0, schlick_r = 0.0;
    int obj = 0;
    const ShadeRec* m = nullptr;
    if (valid && h.key >= 0) {
      const Comps c = prepare(sc, o, d, h);
      hit = true;
      obj = c.obj;
      point = c.point;
      normal = c.normal;
      over = c.over;
      m = &sc.shade[c.obj];
      // reflected_color (world.rs:107-114)
      want_refl = !(req(m->reflective, 0.0) || remaining == 0);
      // refracted_color (world.rs:116-134)
      if (!(req(m->transparency, 0.0) || remaining == 0)) {
        n_ratio = c.n1 / c.n2;
        const double cos_i = vdot(c.eyev, c.normal);
        const double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
        if (!(sin2_t > 1.0)) {
          const double cos_t = sqrt(1.0 - sin2_t);
          k_refr = n_ratio * cos_i - cos_t;
          want_refr = true;
        }
      }
      // shade_hit's Schlick factor (world.rs:62-64), same inputs as the reference's call
      schlick_r = (m->reflective > 0.0 && m->transparency > 0.0) ? schlick(c.eyev, c.normal, c.n1, c.n2) : 0.0;
    }
    V3 surface = v3(0.0, 0.0, 0.0);  // fold from (0,0,0) (color.rs:96-103)
    if (hit) {
      const V3 eyev = vneg(d);  // comps.eyev (intersection.rs:56)
      for (unsigned l = 0; l < L; ++l) {
        cLightRec Lr = (cLightRec)sc.lights + l;
        // the shadow ray exactly as World::is_shadowed builds it (world.rs:95-105); its
        // direction is also lighting()'s light vector (same operands, same operations)
        const V3 v = vsub(v3(Lr->pos[0], Lr->pos[1], Lr->pos[2]), over);
        const double dist = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);  // magnitude (vector.rs:21-23)
        const V3 sdir = v3(v.x / dist, v.y / dist, v.z / dist);       // normalize (vector.rs:25-28)
        V3 term;
        if (a.skip_shadow && shadow_irrelevant(*m, Lr, sdir, normal, term)) {
          // the light is behind the surface: lighting() is the ambient term either way
        } else {
          const bool shadowed = shadow_trace<LANE, QUADS>(sc, a.use_lb, ls, l, over, sdir, dist, tl.sh_disc,
                                                          tl.sh_tests, tl.sh_boxes);
          ++tl.sh_rays;
          term = lighting(*m, Lr, over, eyev, normal, shadowed, sdir);
        }
        surface = vadd(surface, term);
      }
    }
    const unsigned long long c3 = ps_clock<TALLY>();
    // ---- the children: appended to the ring (one reservation per wave),
    // published once every lane's records are in the L2
    const unsigned long long mr = __ballot(want_refl), mf = __ballot(want_refr);
    const unsigned nr = (unsigned)__popcll(mr), nf = (unsigned)__popcll(mf);
    unsigned rb = 0;
    if (nr + nf) {
      if (lane == 0) rb = atomicAdd(&S.tail, nr + nf);
      rb = (unsigned)__builtin_amdgcn_readfirstlane((int)rb);
    }
    const unsigned nk = (want_refl ? 1u : 0u) + (want_refr ? 1u : 0u);
    if (nk) {  // a node with children: its record, its entry in the tree's level list, the child rays
      PsParent* P = par + ((size_t)t * 64u + px) * a.n_int + node;
      ps_st2(P->surface, surface.x, surface.y);
      ps_st2(&P->surface[2], surface.z, schlick_r);
      const ps_u4 tail = {(unsigned)obj, (want_refl ? 1u : 0u) | (want_refr ? 2u : 0u), nk, 0u};
      __builtin_nontemporal_store(tail, (ps_u4*)&P->obj);
      const unsigned li = atomicAdd(&S.lvl[t][g], 1u);
      __builtin_nontemporal_store((uint16_t)((px << 10) | node),
                                  lists + ((size_t)t * (64u * a.n_int) + 64u * ((1u << g) - 1u) + li));
      const unsigned long long below = (1ull << lane) - 1ull;
      if (want_refl) {  // comps.reflectv (intersection.rs:101) from the over point
        PsRay* r = ring + (rb + (unsigned)__popcll(mr & below)) % a.q_cap;
        const V3 rv = vreflect(d, normal);
        ps_st2(&r->o[0], over.x, over.y);
        ps_st2(&r->o[2], over.z, rv.x);
        ps_st2(&r->d[1], rv.y, rv.z);
        __builtin_nontemporal_store((t << 16) | (px << 10) | (2u * node + 1u), &r->id);
      }
      if (want_refr) {  // refracted_color's ray from the under point (world.rs:122-131, intersection.rs:103)
        PsRay* r = ring + (rb + nr + (unsigned)__popcll(mf & below)) % a.q_cap;
        const V3 under = vsub(point, vscale(normal, kEpsilon));
        const V3 refr_dir = vsub(vscale(normal, k_refr), vscale(vneg(d), n_ratio));
        ps_st2(&r->o[0], under.x, under.y);
        ps_st2(&r->o[2], under.z, refr_dir.x);
        ps_st2(&r->d[1], refr_dir.y, refr_dir.z);
        __builtin_nontemporal_store((t << 16) | (px << 10) | (2u * node + 2u), &r->id);
      }
      // the tree gains its children before they become visible (never reaches 0 here)
      atomicAdd(&S.live[t], (int)nk - 1);
    } else if (valid) {  // a node without children: its colour is final (color_at, world.rs:70-81)
      V3 col = v3(0.0, 0.0, 0.0);  // a miss is black (world.rs:74-75)
      if (hit) {
        const V3 zero = v3(0.0, 0.0, 0.0);  // reflected / refracted colour: black (world.rs:108-109, 117-118)
        col = shade_color(*m, surface, zero, zero, schlick_r);
      }
      double* dst;
      if (node == 0u) {
        dst = ps_root_dst(a, cam, S.root0[t] + px);
      } else {  // into its parent's record, for the tree's combine
        PsParent* Q = par + ((size_t)t * 64u + px) * a.n_int + ((node - 1u) >> 1);
        dst = ((node - 1u) & 1u) ? Q->refr : Q->refl;
      }
      ps_st2(dst, col.x, col.y);
      __builtin_nontemporal_store(col.z, dst + 2);
    }
    ps_drain();  // every record, ring entry and colour of this chunk is in the L2
    if (nr + nf && lane == 0) {  // publish in reservation order
      unsigned long long t0 = 0;
      for (unsigned it = 0; ps_ld(&S.commit) != rb; ++it) {
        if ((it & 63u) == 0u) {
          const unsigned long long now = __builtin_amdgcn_s_memrealtime();
          if (it == 0) {
            t0 = now;
          } else if (now - t0 > kPsWaitTicks) {
            ps_fault(a.fault, a.trees, a.q_cap, S, 3, it, now - t0);
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(&S.commit, rb + nr + nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const unsigned long long c4 = ps_clock<TALLY>();
    // ---- a node without children finishes its ray; the lane that finishes a
    // tree's last ray hands the tree to this wave's combine
    bool done_tree = false;
    if (valid && nk == 0u) done_tree = atomicAdd(&S.live[t], -1) == 1;
    unsigned long long md = __ballot(done_tree);
    while (md) {
      const int src = __ffsll((long long)md) - 1;
      const unsigned tt = (unsigned)__shfl((int)t, src, 64);
      ps_combine_tree(sc, a, cam, par, lists, S, tt);
      if (lane == 0) atomicOr(&S.tree_free, 1u << tt);
      md &= md - 1ull;
    }
    const unsigned long long c5 = ps_clock<TALLY>();
    if constexpr (TALLY) {  // counted launch: executed work per class, shade_hit runs and children per depth
      const unsigned cls = kind == PS_ROOTS ? (unsigned)WF_PRIMARY : (unsigned)WF_CLOSEST;
      const unsigned long long s = wave_sum(tl.disc), st = wave_sum(tl.tests), sb = wave_sum(tl.boxes);
      const unsigned long long hs = wave_sum(tl.sh_disc), hst = wave_sum(tl.sh_tests), hsb = wave_sum(tl.sh_boxes);
      const unsigned long long hr = wave_sum(tl.sh_rays);
      if (lane == 0) {
        WfWorkRow* w = cnt->work + ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kWorkRows - 1));
        if (s) atomicAdd(&w->disc[cls], s);
        if (st) atomicAdd(&w->tests[cls], st);
        if (sb) atomicAdd(&w->boxes[cls], sb);
        if (hs) atomicAdd(&w->disc[WF_SHADOW], hs);
        if (hst) { atomicAdd(&w->tests[WF_SHADOW], hst); atomicAdd(&w->sh_tests[cls], hst); }
        if (hsb) atomicAdd(&w->boxes[WF_SHADOW], hsb);
        if (hr) atomicAdd(&w->sh_rays[cls], hr);
        const unsigned q = kind == PS_ROOTS ? 0u : 1u;
        atomicAdd(&w->ps_items[q], 1ull);
        atomicAdd(&w->ps_lanes[q], (unsigned long long)take);
        atomicAdd(&w->ps_cycles[0], c1 - c0);
        atomicAdd(&w->ps_cycles[1], c2 - c1);
        atomicAdd(&w->ps_cycles[2], c3 - c2);
        atomicAdd(&w->ps_cycles[3], c4 - c3);
        atomicAdd(&w->ps_cycles[4], c5 - c4);
      }
      tl = PsTally{};
      if (a.count && valid) {
        if (hit) atomicAdd(&cnt->n_hit[g], 1u);
        if (want_refl) atomicAdd(&cnt->n_refl[g], 1u);
        if (want_refr) atomicAdd(&cnt->n_refr[g], 1u);
      }
    }
    if (lane == 0) atomicSub(&S.busy, 1u);
  }
  // the last workgroup to finish zeroes the frame's counters for the next
  // frame on this workspace (stream order: it runs before the next launch)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned done = atomicAdd(&a.ctr->done, 1u);
    if (done == gridDim.x - 1u) {
      for (unsigned k = 0; k < kPsClasses; ++k) atomicExch(&a.ctr->chunk[k * kPsCtrStride], 0u);
      atomicExch(&a.ctr->done, 0u);
    }
  }
}

// ------------------------------------------------------------------ host side
template <typename K>
static hipError_t ps_launch_k(K kern, unsigned grid, size_t lds, hipStream_t st, hipEvent_t e0, hipEvent_t e1,
                              const DevScene& sc, const DevCamera& cam, const PsArgs& a) {
  hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (e0)
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(kTraceBlock), lds, st, e0, e1, 0, sc, cam, a);
  else
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kTraceBlock), lds, st, sc, cam, a);
  return hipGetLastError();
}

#ifdef RT_PS_LDS_IMAGE
// the LDS image (pair layout): rt_persist_lds.o
hipError_t ps_launch_lds(const DevScene& sc, const DevCamera& cam, const PsArgs& a, bool quads, bool tally,
                         unsigned grid, size_t lds, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (tally)
    return quads ? ps_launch_k(ps_render<14, true, true>, grid, lds, st, e0, e1, sc, cam, a)
                 : ps_launch_k(ps_render<14, false, true>, grid, lds, st, e0, e1, sc, cam, a);
  return quads ? ps_launch_k(ps_render<14, true, false>, grid, lds, st, e0, e1, sc, cam, a)
               : ps_launch_k(ps_render<14, false, false>, grid, lds, st, e0, e1, sc, cam, a);
}
#else
// the global-memory images (image 3: LDS stack + treelet; image 1: scratch stack): rt_persist_glb.o
hipError_t ps_launch_global(const DevScene& sc, const DevCamera& cam, const PsArgs& a, int image, bool quads,
                            bool tally, unsigned grid, size_t lds, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if (image == 3) {
    if (tally)
      return quads ? ps_launch_k(ps_render<3, true, true>, grid, lds, st, e0, e1, sc, cam, a)
                   : ps_launch_k(ps_render<3, false, true>, grid, lds, st, e0, e1, sc, cam, a);
    return quads ? ps_launch_k(ps_render<3, true, false>, grid, lds, st, e0, e1, sc, cam, a)
                 : ps_launch_k(ps_render<3, false, false>, grid, lds, st, e0, e1, sc, cam, a);
  }
  if (tally)
    return quads ? ps_launch_k(ps_render<1, true, true>, grid, lds, st, e0, e1, sc, cam, a)
                 : ps_launch_k(ps_render<1, false, true>, grid, lds, st, e0, e1, sc, cam, a);
  return quads ? ps_launch_k(ps_render<1, true, false>, grid, lds, st, e0, e1, sc, cam, a)
               : ps_launch_k(ps_render<1, false, false>, grid, lds, st, e0, e1, sc, cam, a);
}
#endif

}  // namespace rtamd
