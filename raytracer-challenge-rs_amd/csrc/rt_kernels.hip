// rt_kernels.hip — MI355X (gfx950) kernels for the per-pixel render path of
// tlinford/raytracer-challenge-rs: `Camera::render` (camera.rs:133-148) ->
// `World::color_at` (world.rs:70-81) -> intersect / hit / prepare_computations /
// shade_hit / lighting / is_shadowed / reflected_color / refracted_color.
//
// Design (DESIGN.md "Kernel"):
//  * One lane = one pixel's whole recursion tree, evaluated depth-first with an
//    explicit per-lane stack in scratch. The stack reproduces the reference's
//    post-order combine exactly: surface (left fold over lights), then
//    reflected, then refracted, combined as (surface + refl) + refr or with the
//    Schlick weights (world.rs:40-68). No path-weight re-association.
//  * Persistent waves: a lane whose tree is finished takes the next pixel from
//    a global counter (one atomic per wave per refill), so every trace step
//    runs with (almost) all 64 lanes busy, whatever the tree sizes.
//  * Every trace step tests every shape (the reference's brute-force
//    `World::intersect`). Shape records are wave-uniform: they are read with
//    scalar loads (s_load) from the constant address space and feed the f64
//    VALU as SGPR operands; no LDS and no per-lane shape loads in the hot loop.
//  * Nearest hit without the sorted list: min over (t, key) with key =
//    2*object + root (the stable-sort order of the reference's list).
//    `containers` (intersection.rs:63-90) is replaced by the exact top-2
//    formulation over the strictly-negative roots (DESIGN.md "n1/n2").
//  * All arithmetic is binary64 in the reference's operation order; the file
//    is compiled with -ffp-contract=off and also pins `fp contract(off)`.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rt_device.hpp"
#include "rt_kernels.hpp"

#pragma clang fp contract(off)

namespace rtamd {

// --------------------------------------------------------------- the stack
struct Frame {
  V3 over, under, eyev, normal;
  V3 surf;  // running sum over lights (world.rs:41-56)
  V3 refl;  // reflected_color(...) already multiplied by `reflective`
  double n1, n2;
  int obj, light, phase, pad;
};
enum : int { PH_AWAIT_REFL = 1, PH_AWAIT_REFR = 2 };
enum : int { OP_NEXT_LIGHT = 0, OP_REFLECT = 1, OP_REFRACT = 2, OP_FINISH = 3, OP_RETURN = 4 };

template <int MAXF, bool FROM_RAYS, int BLOCK, int WAVES, bool USE_LDS, bool DIAG = false>
__global__ __launch_bounds__(BLOCK, WAVES) void render_kernel(DevScene sc, DevCamera cam, RenderArgs args) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  unsigned long long diag_t0 = 0, diag_trace = 0, wave_steps = 0;
  if constexpr (DIAG) diag_t0 = __builtin_amdgcn_s_memtime();
  LdsView lv{};
  if constexpr (USE_LDS) lv = lds_stage(sc, lds_raw);
  Frame stk[MAXF];
  const int lane = threadIdx.x & 63;
  int task = -1;  // pixel (render) or ray (batch) index, -1 = idle
  int depth = 0;
  V3 ro = v3(0, 0, 0), rd = v3(0, 0, 0);
  bool shadow_mode = false;
  double sdist = 0.0;
  unsigned n_prim = 0, n_refl = 0, n_refr = 0, n_shadow = 0, n_traces = 0;
  unsigned n_disc = 0;
  bool no_more = false;
  cLightRec lights = (cLightRec)sc.lights;

  while (true) {
    // ---- refill idle lanes: one atomic per wave (wave-uniform control flow)
    if (!no_more) {
      const unsigned long long want = __ballot(task < 0);
      if (want) {
        const unsigned cnt = (unsigned)__popcll(want);
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(args.counter, cnt);
        base = __shfl(base, 0, 64);
        if (task < 0) {
          const unsigned rank = (unsigned)__popcll(want & ((1ull << lane) - 1ull));
          const unsigned my = base + rank;
          if (my < args.n_tasks) {
            task = (int)my;
            depth = 0;
            shadow_mode = false;
            ++n_prim;
            if constexpr (FROM_RAYS) {
              const double* r = args.rays + (size_t)my * 6;
              ro = v3(r[0], r[1], r[2]);
              rd = v3(r[3], r[4], r[5]);
            } else {
              // shard row mapping: local row lr -> global row y
              const uint32_t lr = my / cam.hsize, x = my - lr * cam.hsize;
              const uint32_t blk = lr / args.row_block, off = lr - blk * args.row_block;
              const uint32_t y = (blk * args.n_shards + args.shard) * args.row_block + off;
              ray_for_pixel(cam, x, y, ro, rd);
            }
          }
        }
        if (base + cnt >= args.n_tasks) no_more = true;
      }
    }
    if (__ballot(task >= 0) == 0ull) break;
    ++wave_steps;
    unsigned long long diag_s0 = 0;
    if constexpr (DIAG) diag_s0 = __builtin_amdgcn_s_memtime();
    if (task < 0) continue;

    // ---- one trace per active lane (all lanes walk the same shape stream)
    Hit h;
    trace<USE_LDS>(sc, lv, ro, rd, shadow_mode, h, n_disc);
    ++n_traces;
    if constexpr (DIAG) diag_trace += __builtin_amdgcn_s_memtime() - diag_s0;

    // ---- advance this lane's recursion until it needs the next trace
    int op;
    V3 ret = v3(0.0, 0.0, 0.0);
    V3 refr = v3(0.0, 0.0, 0.0);
    if (shadow_mode) {
      // World::is_shadowed (world.rs:95-105): first shadow-casting t >= 0 < distance
      Frame& f = stk[depth];
      const bool shadowed = h.key >= 0 && h.t < sdist;
      const ShadeRec& m = sc.shade[f.obj];
      const V3 c = lighting(m, lights + f.light, f.over, f.eyev, f.normal, shadowed);
      f.surf = vadd(f.surf, c);
      f.light += 1;
      op = OP_NEXT_LIGHT;
    } else if (h.key < 0) {
      ret = v3(0.0, 0.0, 0.0);  // miss -> Color::black() (world.rs:74-75)
      op = OP_RETURN;
    } else {
      const Comps c = prepare(sc, ro, rd, h);
      Frame& f = stk[depth];
      f.over = c.over; f.under = c.under; f.eyev = c.eyev; f.normal = c.normal;
      f.n1 = c.n1; f.n2 = c.n2; f.obj = c.obj;
      f.surf = v3(0.0, 0.0, 0.0);  // Sum starts from (0,0,0) (color.rs:96-103)
      f.light = 0;
      op = OP_NEXT_LIGHT;
    }
    bool need_trace = false;
    while (!need_trace && task >= 0) {
      Frame& f = stk[depth];
      if (op == OP_NEXT_LIGHT) {
        if (f.light < sc.n_lights) {
          cLightRec L = lights + f.light;
          const V3 v = vsub(v3(L->pos[0], L->pos[1], L->pos[2]), f.over);
          sdist = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);  // magnitude
          rd = vnormalize(v);
          ro = f.over;
          shadow_mode = true;
          ++n_shadow;
          need_trace = true;
        } else {
          op = OP_REFLECT;
        }
      } else if (op == OP_REFLECT) {
        // World::reflected_color (world.rs:107-114)
        const ShadeRec& m = sc.shade[f.obj];
        const uint32_t remaining = args.max_depth - (uint32_t)depth;
        if (req(m.reflective, 0.0) || remaining == 0) {
          f.refl = v3(0.0, 0.0, 0.0);
          op = OP_REFRACT;
        } else {
          f.phase = PH_AWAIT_REFL;
          const V3 d = vneg(f.eyev);  // the incoming direction, exactly
          ro = f.over;
          rd = vreflect(d, f.normal);  // comps.reflectv (intersection.rs:101)
          shadow_mode = false;
          ++depth;
          ++n_refl;
          need_trace = true;
        }
      } else if (op == OP_REFRACT) {
        // World::refracted_color (world.rs:116-134)
        const ShadeRec& m = sc.shade[f.obj];
        const uint32_t remaining = args.max_depth - (uint32_t)depth;
        refr = v3(0.0, 0.0, 0.0);
        op = OP_FINISH;
        if (!(req(m.transparency, 0.0) || remaining == 0)) {
          const double n_ratio = f.n1 / f.n2;
          const double cos_i = vdot(f.eyev, f.normal);
          const double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
          if (!(sin2_t > 1.0)) {
            const double cos_t = sqrt(1.0 - sin2_t);
            rd = vsub(vscale(f.normal, n_ratio * cos_i - cos_t), vscale(f.eyev, n_ratio));
            ro = f.under;
            f.phase = PH_AWAIT_REFR;
            shadow_mode = false;
            ++depth;
            ++n_refr;
            need_trace = true;
          }
        }
      } else if (op == OP_FINISH) {
        // world.rs:61-67
        const ShadeRec& m = sc.shade[f.obj];
        if (m.reflective > 0.0 && m.transparency > 0.0) {
          const double r = schlick(f.eyev, f.normal, f.n1, f.n2);
          ret = vadd(vadd(f.surf, vscale(f.refl, r)), vscale(refr, 1.0 - r));
        } else {
          ret = vadd(vadd(f.surf, f.refl), refr);
        }
        op = OP_RETURN;
      } else {  // OP_RETURN: hand `ret` to the parent frame
        if (depth == 0) {
          double* out = args.out + (size_t)task * 3;
          out[0] = ret.x; out[1] = ret.y; out[2] = ret.z;
          task = -1;
        } else {
          --depth;
          Frame& p = stk[depth];
          const ShadeRec& m = sc.shade[p.obj];
          if (p.phase == PH_AWAIT_REFL) {
            p.refl = vscale(ret, m.reflective);  // world.rs:113
            op = OP_REFRACT;
          } else {
            refr = vscale(ret, m.transparency);  // world.rs:133
            op = OP_FINISH;
          }
        }
      }
    }
  }

  // ---- counters: one atomic per wave per field
  const unsigned long long s_prim = wave_sum(n_prim), s_refl = wave_sum(n_refl);
  const unsigned long long s_refr = wave_sum(n_refr), s_shadow = wave_sum(n_shadow);
  const unsigned long long s_tr = wave_sum(n_traces), s_disc = wave_sum(n_disc);
  if (lane == 0 && args.stats) {
    atomicAdd(&args.stats->rays_primary, s_prim);
    atomicAdd(&args.stats->rays_reflect, s_refl);
    atomicAdd(&args.stats->rays_refract, s_refr);
    atomicAdd(&args.stats->rays_shadow, s_shadow);
    atomicAdd(&args.stats->sphere_tests, s_tr * (unsigned long long)(sc.n_diag + sc.n_gen));
    atomicAdd(&args.stats->plane_tests, s_tr * (unsigned long long)sc.n_planes);
    atomicAdd(&args.stats->sphere_disc_ge0, s_disc);
    atomicAdd(&args.stats->wave_steps, wave_steps);
    if constexpr (DIAG) {
      atomicAdd(&args.stats->diag_trace_cycles, diag_trace);
      atomicAdd(&args.stats->diag_total_cycles, __builtin_amdgcn_s_memtime() - diag_t0);
    }
  }
}

// rt_hit_batch: World::intersect + hit + prepare_computations + schlick per ray.
__global__ __launch_bounds__(256) void hit_kernel(DevScene sc, const double* rays, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3 o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
  const V3 d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
  Hit h;
  unsigned nd = 0;
  trace<false>(sc, LdsView{}, o, d, false, h, nd);
  double* r = out + (size_t)i * 24;
  for (int k = 0; k < 24; ++k) r[k] = 0.0;
  r[0] = -1.0;
  if (h.key < 0) return;
  const Comps c = prepare(sc, o, d, h);
  r[0] = c.obj; r[1] = h.t;
  r[2] = c.point.x; r[3] = c.point.y; r[4] = c.point.z;
  r[5] = c.over.x; r[6] = c.over.y; r[7] = c.over.z;
  r[8] = c.under.x; r[9] = c.under.y; r[10] = c.under.z;
  r[11] = c.eyev.x; r[12] = c.eyev.y; r[13] = c.eyev.z;
  r[14] = c.normal.x; r[15] = c.normal.y; r[16] = c.normal.z;
  r[17] = c.inside ? 1.0 : 0.0;
  const V3 rv = vreflect(d, c.normal);
  r[18] = rv.x; r[19] = rv.y; r[20] = rv.z;
  r[21] = c.n1; r[22] = c.n2;
  r[23] = schlick(c.eyev, c.normal, c.n1, c.n2);
}

// rt_is_shadowed_batch: World::is_shadowed for each point against one light.
__global__ __launch_bounds__(256) void shadow_kernel(DevScene sc, const double* pts, int n, int light,
                                                     uint8_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3 p = v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
  const LightRec L = sc.lights[light];
  const V3 v = vsub(v3(L.pos[0], L.pos[1], L.pos[2]), p);
  const double distance = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
  const V3 d = vnormalize(v);
  Hit h;
  unsigned nd = 0;
  trace<false>(sc, LdsView{}, p, d, true, h, nd);
  out[i] = (h.key >= 0 && h.t < distance) ? 1 : 0;
}

// ------------------------------------------------------------ host launchers
template <int MAXF, bool FROM_RAYS, int BLOCK, int WAVES, bool USE_LDS, bool DIAG = false>
static hipError_t launch_render_w(const DevScene& sc, const DevCamera& cam, const RenderArgs& args,
                                  hipStream_t stream) {
  auto kern = render_kernel<MAXF, FROM_RAYS, BLOCK, WAVES, USE_LDS, DIAG>;
  const size_t lds = USE_LDS ? lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes) : 0;
  hipError_t e;
  if (USE_LDS) {
    e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  int dev = 0;
  e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  int n_cu = 0;
  e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  int per_cu = 0;
  e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BLOCK, lds);
  if (e != hipSuccess || per_cu < 1) per_cu = 1;
  long long want = ((long long)args.n_tasks + BLOCK - 1) / BLOCK;
  long long cap = (long long)n_cu * per_cu;
  if (args.grid_cap > 0 && args.grid_cap < cap) cap = args.grid_cap;
  long long grid = want < cap ? want : cap;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(BLOCK), lds, stream, sc, cam, args);
  return hipGetLastError();
}

// LDS staging when the whole record list fits in one CU's LDS (one 768-thread
// workgroup per CU = 3 waves per SIMD, one copy per CU), else scalar loads.
constexpr size_t kLdsLimit = 160 * 1024 - 1024;

// Variants (RenderArgs::waves, tuning knob): 0 = default (LDS if it fits).
template <int MAXF, bool FROM_RAYS>
static hipError_t launch_render_t(const DevScene& sc, const DevCamera& cam, const RenderArgs& a,
                                  hipStream_t s) {
  const bool fits = lds_bytes(sc.n_diag, sc.n_gen, sc.n_planes) <= kLdsLimit;
  switch (a.waves) {
    case 3: return launch_render_w<MAXF, FROM_RAYS, 256, 3, false>(sc, cam, a, s);
    case 4: return launch_render_w<MAXF, FROM_RAYS, 256, 4, false>(sc, cam, a, s);
    case 20:  // diagnostic build: s_memtime around every trace step (never the default)
      if (fits && !FROM_RAYS) return launch_render_w<MAXF, FROM_RAYS, 768, 3, true, true>(sc, cam, a, s);
      return launch_render_w<MAXF, FROM_RAYS, 256, kDefaultWaves, false, true>(sc, cam, a, s);
    default:
      if (fits && !FROM_RAYS) return launch_render_w<MAXF, FROM_RAYS, 768, 3, true>(sc, cam, a, s);
      return launch_render_w<MAXF, FROM_RAYS, 256, kDefaultWaves, false>(sc, cam, a, s);
  }
}

template <bool FROM_RAYS>
static hipError_t launch_render_depth(const DevScene& sc, const DevCamera& cam, const RenderArgs& a,
                                      hipStream_t s) {
  if (a.max_depth <= 5) return launch_render_t<6, FROM_RAYS>(sc, cam, a, s);
  if (a.max_depth <= 8) return launch_render_t<9, FROM_RAYS>(sc, cam, a, s);
  if (a.max_depth <= 16) return launch_render_t<17, FROM_RAYS>(sc, cam, a, s);
  return launch_render_t<kMaxDepth + 1, FROM_RAYS>(sc, cam, a, s);
}

hipError_t launch_render(const DevScene& sc, const DevCamera& cam, const RenderArgs& args,
                         hipStream_t stream) {
  if (args.rays) return launch_render_depth<true>(sc, cam, args, stream);
  return launch_render_depth<false>(sc, cam, args, stream);
}

hipError_t launch_hit(const DevScene& sc, const double* d_rays, int n, double* d_out, hipStream_t s) {
  hipLaunchKernelGGL(hit_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sc, d_rays, n, d_out);
  return hipGetLastError();
}

hipError_t launch_shadow(const DevScene& sc, const double* d_pts, int n, int light, uint8_t* d_out,
                         hipStream_t s) {
  hipLaunchKernelGGL(shadow_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sc, d_pts, n, light, d_out);
  return hipGetLastError();
}

}  // namespace rtamd
