// rt_wf_combine.hip — the wavefront frame's kernels besides the trace
// launches: wf_frame_init (counters, primary records, the batch's camera
// table), wf_prep / wf_combine (the exhaustive pipeline's shading and
// `shade_hit` sum), wf_combine_parents (the fast path's `shade_hit` sum for
// nodes with children, world.rs:40-68, deepest generation first), wf_average
// (`Color::average` of AA samples, color.rs:26-33) and wf_count_kinds.
#include "rt_wf_device.hpp"

#pragma clang fp contract(off)

namespace rtamd {

// ------------------------------------------------------------ primary records
// Per diagonal sphere: s (inverse diagonal), o' = s*o + t for the camera origin
// o, and c = o'.o' - 1 — the same operations the general test performs, so the
// values are bit-identical to what each primary ray would compute.
// The frame's first launch: zero the work counters and the queue counters of
// this workspace (n_a and n_b 16-B words) and, for a camera frame, write the
// primary records (wf_prim_prep's computation). One launch instead of two
// fills and a kernel.
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


}  // namespace rtamd
