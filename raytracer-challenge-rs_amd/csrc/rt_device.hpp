// rt_device.hpp — device-side building blocks of the render path, shared by
// the persistent megakernel (rt_kernels.hip) and the wavefront pipeline
// (rt_wavefront.hip). Every function restates a reference function (cited),
// in binary64 with the reference's operation order; include only from .hip
// files compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rt_layout.hpp"

#pragma clang fp contract(off)

namespace rtamd {

// --------------------------------------------------------------- vector math
// vector.rs / point.rs / color.rs, left-associative like the Rust expressions.
struct V3 {
  double x, y, z;
};
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 vscale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
// vector.rs:99-101
__device__ __forceinline__ double vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vector.rs:21-28 (three divisions, not a reciprocal)
__device__ __forceinline__ V3 vnormalize(V3 a) {
  double m = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  return v3(a.x / m, a.y / m, a.z / m);
}
// vector.rs:30-32: self - normal * 2.0 * dot(self, normal)
__device__ __forceinline__ V3 vreflect(V3 v, V3 n) { return vsub(v, vscale(vscale(n, 2.0), vdot(v, n))); }
// lib.rs:20-22
__device__ __forceinline__ bool req(double a, double b) { return fabs(a - b) < kEpsilon; }
// matrix.rs:232-245 (point, rows 0..2 with translation) and :247-260 (vector)
__device__ __forceinline__ V3 m34_point(const double* m, V3 p) {
  return v3(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3],
            m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
            m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
__device__ __forceinline__ V3 m33_vector(const double* m, V3 v) {  // m: 3x3 row-major
  return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z,
            m[3] * v.x + m[4] * v.y + m[5] * v.z,
            m[6] * v.x + m[7] * v.y + m[8] * v.z);
}

// Wave-uniform records through the constant address space -> s_load.
#define RT_CONST __attribute__((address_space(4)))
typedef const RT_CONST SphereDiag* cSphereDiag;
typedef const RT_CONST SphereGen* cSphereGen;
typedef const RT_CONST PlaneRec* cPlaneRec;
typedef const RT_CONST LightRec* cLightRec;

// ------------------------------------------------------------ trace (hot loop)
struct Hit {
  double t;   // nearest t >= 0 (over eligible objects)
  int key;    // 2*object + root, -1 = miss
  // containers candidates (radiance rays): top-2 by (entry t, key) among
  // spheres with t1 < 0 <= t2 and planes with t < 0.
  double c1t, c2t;
  int c1k, c2k;
};

__device__ __forceinline__ bool better(double t, int k, double bt, int bk) {
  return t < bt || (t == bt && k < bk);
}
__device__ __forceinline__ void push_container(Hit& h, double t, int k) {
  if (t > h.c1t || (t == h.c1t && k > h.c1k)) {
    h.c2t = h.c1t; h.c2k = h.c1k; h.c1t = t; h.c1k = k;
  } else if (t > h.c2t || (t == h.c2t && k > h.c2k)) {
    h.c2t = t; h.c2k = k;
  }
}

// Sphere::local_intersect (sphere.rs:47-62) on the object-space ray.
// With b = 2*dt and disc = b*b - (4a)*c = 4*(dt*dt - a*c) exactly (power-of-two
// scaling commutes with rounding), t = (-b -/+ sqrt(disc)) / (2a) equals
// (-dt -/+ sqrt(dt*dt - a*c)) / a bit for bit (DESIGN.md "Sphere roots").
__device__ __forceinline__ void sphere_roots(double ox, double oy, double oz, double dx, double dy,
                                             double dz, int64_t meta, bool shadow_mode, Hit& h,
                                             unsigned& n_disc) {
  const double a = dx * dx + dy * dy + dz * dz;
  const double dt = dx * ox + dy * oy + dz * oz;
  const double c = ox * ox + oy * oy + oz * oz - 1.0;
  const double disc = dt * dt - a * c;
  if (disc >= 0.0) {
    ++n_disc;
    const double q = sqrt(disc);
    const double t1 = (-dt - q) / a;
    const double t2 = (-dt + q) / a;
    const int k1 = (int)(meta >> 1) * 2;
    const bool eligible = !shadow_mode || (meta & 1);
    if (eligible) {
      if (t1 >= 0.0) {
        if (better(t1, k1, h.t, h.key)) { h.t = t1; h.key = k1; }
      } else if (t2 >= 0.0) {
        if (better(t2, k1 + 1, h.t, h.key)) { h.t = t2; h.key = k1 + 1; }
      }
    }
    if (t1 < 0.0 && t2 >= 0.0) push_container(h, t1, k1);
  }
}

// Same test with the object index / shadow flag fetched only when the
// discriminant is non-negative (LDS path: the meta word is not needed per test).
__device__ __forceinline__ void sphere_roots_lazy(double ox, double oy, double oz, double dx, double dy,
                                                  double dz, const int* meta_p, bool shadow_mode, Hit& h,
                                                  unsigned& n_disc) {
  const double a = dx * dx + dy * dy + dz * dz;
  const double dt = dx * ox + dy * oy + dz * oz;
  const double c = ox * ox + oy * oy + oz * oz - 1.0;
  const double disc = dt * dt - a * c;
  if (disc >= 0.0) {
    ++n_disc;
    const int meta = *meta_p;
    const double q = sqrt(disc);
    const double t1 = (-dt - q) / a;
    const double t2 = (-dt + q) / a;
    const int k1 = (meta >> 1) * 2;
    const bool eligible = !shadow_mode || (meta & 1);
    if (eligible) {
      if (t1 >= 0.0) {
        if (better(t1, k1, h.t, h.key)) { h.t = t1; h.key = k1; }
      } else if (t2 >= 0.0) {
        if (better(t2, k1 + 1, h.t, h.key)) { h.t = t2; h.key = k1 + 1; }
      }
    }
    if (t1 < 0.0 && t2 >= 0.0) push_container(h, t1, k1);
  }
}

// LDS image of the trace records (one copy per workgroup = per CU):
//   diag: 6 doubles (s0 s1 s2 t0 t1 t2) per sphere, gen: 12 doubles, plane: 4
//   doubles; then int32 meta arrays. Reads are wave-uniform (broadcast).
struct LdsView {
  const double* diag;
  const double* gen;
  const double* plane;
  const int* diag_meta;
  const int* gen_meta;
  const int* plane_meta;
};
typedef double d2 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr size_t lds_align16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline size_t lds_bytes(int nd, int ng, int np) {
  return lds_align16((size_t)(nd + 4) * 48) + lds_align16((size_t)ng * 96) + lds_align16((size_t)np * 32) +
         lds_align16((size_t)nd * 4) + lds_align16((size_t)ng * 4) + lds_align16((size_t)np * 4);
}

__device__ LdsView lds_stage(const DevScene& sc, unsigned char* base) {
  LdsView v;
  size_t off = 0;
  v.diag = (const double*)(base + off); off += lds_align16((size_t)(sc.n_diag + 4) * 48);
  v.gen = (const double*)(base + off); off += lds_align16((size_t)sc.n_gen * 96);
  v.plane = (const double*)(base + off); off += lds_align16((size_t)sc.n_planes * 32);
  v.diag_meta = (const int*)(base + off); off += lds_align16((size_t)sc.n_diag * 4);
  v.gen_meta = (const int*)(base + off); off += lds_align16((size_t)sc.n_gen * 4);
  v.plane_meta = (const int*)(base + off);
  double* dd = (double*)v.diag;
  double* dg = (double*)v.gen;
  double* dp = (double*)v.plane;
  for (int i = threadIdx.x; i < (sc.n_diag + 4) * 6; i += blockDim.x) {
    const int r = i / 6, e = i - r * 6;
    dd[i] = r >= sc.n_diag ? 0.0 : e < 3 ? sc.sph_diag[r].s[e] : sc.sph_diag[r].t[e - 3];
  }
  for (int i = threadIdx.x; i < sc.n_gen * 12; i += blockDim.x) dg[i] = sc.sph_gen[i / 12].m[i % 12];
  for (int i = threadIdx.x; i < sc.n_planes * 4; i += blockDim.x) dp[i] = sc.planes[i / 4].m[i % 4];
  for (int i = threadIdx.x; i < sc.n_diag; i += blockDim.x) ((int*)v.diag_meta)[i] = (int)sc.sph_diag[i].meta;
  for (int i = threadIdx.x; i < sc.n_gen; i += blockDim.x) ((int*)v.gen_meta)[i] = (int)sc.sph_gen[i].meta;
  for (int i = threadIdx.x; i < sc.n_planes; i += blockDim.x) ((int*)v.plane_meta)[i] = (int)sc.planes[i].meta;
  __syncthreads();
  return v;
}

// World::intersect + hit (world.rs:31-38, intersection.rs:118-125): every
// object, in three wave-uniform record streams.
template <bool USE_LDS>
__device__ __forceinline__ void trace(const DevScene& sc, const LdsView& lv, V3 o, V3 d, bool shadow_mode,
                                      Hit& h, unsigned& n_disc) {
  h.t = INFINITY;
  h.c1t = -INFINITY; h.c2t = -INFINITY; h.c1k = -1; h.c2k = -1;
  h.key = 0x7fffffff;
  // Shape::intersect (geometry/mod.rs:46-49): Ray::transform by the inverse.
  if constexpr (USE_LDS) {
    if (sc.n_diag > 0) {
      // ping-pong look-ahead from LDS (3 x ds_read_b128 per record, broadcast);
      // the image holds zero padding records, so record j+1 always exists.
      // record layout: (s0 s1) (s2 t0) (t1 t2); off-diagonal inverse entries are exact zeros
      const d2* r = (const d2*)lv.diag;
      d2 a0 = r[0], a1 = r[1], a2 = r[2];
      int j = 0;
      for (; j + 1 < sc.n_diag; j += 2) {
        const d2 b0 = r[3 * j + 3], b1 = r[3 * j + 4], b2 = r[3 * j + 5];
        sphere_roots_lazy(a0.x * o.x + a1.y, a0.y * o.y + a2.x, a1.x * o.z + a2.y, a0.x * d.x, a0.y * d.y,
                          a1.x * d.z, lv.diag_meta + j, shadow_mode, h, n_disc);
        a0 = r[3 * j + 6]; a1 = r[3 * j + 7]; a2 = r[3 * j + 8];
        sphere_roots_lazy(b0.x * o.x + b1.y, b0.y * o.y + b2.x, b1.x * o.z + b2.y, b0.x * d.x, b0.y * d.y,
                          b1.x * d.z, lv.diag_meta + j + 1, shadow_mode, h, n_disc);
      }
      if (j < sc.n_diag)
        sphere_roots_lazy(a0.x * o.x + a1.y, a0.y * o.y + a2.x, a1.x * o.z + a2.y, a0.x * d.x, a0.y * d.y,
                          a1.x * d.z, lv.diag_meta + j, shadow_mode, h, n_disc);
    }
  } else {
    cSphereDiag sd = (cSphereDiag)sc.sph_diag;
    if (sc.n_diag > 0) {
      // software pipeline: the scalar loads of record j+1 are in flight while
      // record j is tested (each section ends with one padding record, so the
      // look-ahead load is always in bounds)
      double s0 = sd[0].s[0], s1 = sd[0].s[1], s2 = sd[0].s[2];
      double t0 = sd[0].t[0], t1 = sd[0].t[1], t2 = sd[0].t[2];
      int64_t meta = sd[0].meta;
      for (int j = 0; j < sc.n_diag; ++j) {
        const double n_s0 = sd[j + 1].s[0], n_s1 = sd[j + 1].s[1], n_s2 = sd[j + 1].s[2];
        const double n_t0 = sd[j + 1].t[0], n_t1 = sd[j + 1].t[1], n_t2 = sd[j + 1].t[2];
        const int64_t n_meta = sd[j + 1].meta;
        // off-diagonal entries are exact zeros: ((m00*x + 0) + 0) + m03 == m00*x + m03
        sphere_roots(s0 * o.x + t0, s1 * o.y + t1, s2 * o.z + t2, s0 * d.x, s1 * d.y, s2 * d.z, meta,
                     shadow_mode, h, n_disc);
        s0 = n_s0; s1 = n_s1; s2 = n_s2; t0 = n_t0; t1 = n_t1; t2 = n_t2; meta = n_meta;
      }
    }
  }
  for (int j = 0; j < sc.n_gen; ++j) {
    double m[12];
    if constexpr (USE_LDS) {
#pragma unroll
      for (int e = 0; e < 12; ++e) m[e] = lv.gen[12 * j + e];
    } else {
      cSphereGen sg = (cSphereGen)sc.sph_gen;
#pragma unroll
      for (int e = 0; e < 12; ++e) m[e] = sg[j].m[e];
    }
    const V3 lo = m34_point(m, o);
    const V3 ld = v3(m[0] * d.x + m[1] * d.y + m[2] * d.z, m[4] * d.x + m[5] * d.y + m[6] * d.z,
                     m[8] * d.x + m[9] * d.y + m[10] * d.z);
    if constexpr (USE_LDS) {
      sphere_roots_lazy(lo.x, lo.y, lo.z, ld.x, ld.y, ld.z, lv.gen_meta + j, shadow_mode, h, n_disc);
    } else {
      sphere_roots(lo.x, lo.y, lo.z, ld.x, ld.y, ld.z, ((cSphereGen)sc.sph_gen)[j].meta, shadow_mode, h, n_disc);
    }
  }
  // Plane::local_intersect (plane.rs:53-60): only object-space y matters.
  for (int j = 0; j < sc.n_planes; ++j) {
    double m0, m1, m2, m3;
    int meta;
    if constexpr (USE_LDS) {
      m0 = lv.plane[4 * j]; m1 = lv.plane[4 * j + 1]; m2 = lv.plane[4 * j + 2]; m3 = lv.plane[4 * j + 3];
      meta = lv.plane_meta[j];
    } else {
      cPlaneRec pl = (cPlaneRec)sc.planes;
      m0 = pl[j].m[0]; m1 = pl[j].m[1]; m2 = pl[j].m[2]; m3 = pl[j].m[3];
      meta = (int)pl[j].meta;
    }
    const double oy = m0 * o.x + m1 * o.y + m2 * o.z + m3;
    const double dy = m0 * d.x + m1 * d.y + m2 * d.z;
    if (!(fabs(dy) < kEpsilon)) {
      const double t = -oy / dy;
      const int k = (meta >> 1) * 2;
      const bool eligible = !shadow_mode || (meta & 1);
      if (eligible && t >= 0.0 && better(t, k, h.t, h.key)) { h.t = t; h.key = k; }
      if (t < 0.0) push_container(h, t, k);
    }
  }
  if (h.key == 0x7fffffff) h.key = -1;
}

// --------------------------------------------------------------- shading
struct Comps {
  V3 point, over, under, eyev, normal;
  double n1, n2;
  int obj;
  bool inside;
};

// Intersection::prepare_computations (intersection.rs:53-105) with the exact
// top-2 replacement of the containers walk.
__device__ __forceinline__ Comps prepare(const DevScene& sc, V3 o, V3 d, const Hit& h) {
  Comps c;
  const int obj = h.key >> 1;
  const ShadeRec& s = sc.shade[obj];
  c.obj = obj;
  c.point = vadd(o, vscale(d, h.t));  // ray.rs:22-24
  c.eyev = vneg(d);
  // Shape::normal_at (geometry/mod.rs:51-56)
  const V3 lp = m34_point(s.inv, c.point);
  const V3 ln = s.kind == 0 ? vsub(lp, v3(0.0, 0.0, 0.0)) : v3(0.0, 1.0, 0.0);
  V3 n = vnormalize(m33_vector(s.invT, ln));
  c.inside = false;
  if (vdot(n, c.eyev) < 0.0) { c.inside = true; n = vneg(n); }
  c.normal = n;
  // n1 / n2 (intersection.rs:63-90, DESIGN.md "n1/n2")
  const bool hit_is_container = (h.key & 1) != 0;  // exit root of a sphere whose t1 < 0
  c.n1 = h.c1k >= 0 ? sc.shade[h.c1k >> 1].refractive_index : 1.0;
  if (!hit_is_container) {
    c.n2 = s.refractive_index;
  } else if ((h.c1k >> 1) == obj) {
    c.n2 = h.c2k >= 0 ? sc.shade[h.c2k >> 1].refractive_index : 1.0;
  } else {
    c.n2 = sc.shade[h.c1k >> 1].refractive_index;
  }
  c.over = vadd(c.point, vscale(n, kEpsilon));
  c.under = vsub(c.point, vscale(n, kEpsilon));
  return c;
}

// Computations::schlick (intersection.rs:147-162); powi(2) = q*q,
// powi(5) = x*((x*x)*(x*x)) (LLVM powi expansion / __powidf2).
__device__ __forceinline__ double schlick(V3 eyev, V3 normal, double n1, double n2) {
  double cosv = vdot(eyev, normal);
  if (n1 > n2) {
    const double nn = n1 / n2;
    const double sin2_t = nn * nn * (1.0 - cosv * cosv);
    if (sin2_t > 1.0) return 1.0;
    cosv = sqrt(1.0 - sin2_t);
  }
  const double q = (n1 - n2) / (n1 + n2);
  const double r0 = q * q;
  const double x = 1.0 - cosv;
  const double x5 = x * ((x * x) * (x * x));
  return r0 + (1.0 - r0) * x5;
}

// Pattern::color_at_shape (pattern/mod.rs:39-49) and the five kinds.
__device__ __forceinline__ V3 pattern_color(const ShadeRec& s, V3 world_point) {
  const V3 op = m34_point(s.inv, world_point);
  const V3 pp = m34_point(s.pat_inv, op);
  const V3 a = v3(s.pat_a[0], s.pat_a[1], s.pat_a[2]);
  const V3 b = v3(s.pat_b[0], s.pat_b[1], s.pat_b[2]);
  switch (s.pattern_kind) {
    case 0:  // test_pattern.rs:7-9
      return pp;
    case 1:  // stripe.rs:14-20
      return fmod(floor(pp.x), 2.0) == 0.0 ? a : b;
    case 2: {  // gradient.rs:14-18
      const V3 distance = vsub(b, a);
      const double fraction = pp.x - floor(pp.x);
      return vadd(a, vscale(distance, fraction));
    }
    case 3: {  // ring.rs:14-21
      const double distance = floor(sqrt(pp.x * pp.x + pp.z * pp.z));
      return fmod(distance, 2.0) == 0.0 ? a : b;
    }
    default: {  // checkers.rs:14-21: `as isize` (saturating) then % 2
      const double distance = floor(pp.x) + floor(pp.y) + floor(pp.z);
      bool even;
      if (isnan(distance)) even = true;                          // NaN as isize = 0
      else if (distance >= 9223372036854775808.0) even = false;  // isize::MAX is odd
      else if (distance < -9223372036854775808.0) even = true;   // isize::MIN is even
      else even = fmod(distance, 2.0) == 0.0;                   // exact integer parity
      return even ? a : b;
    }
  }
}

// Material::lighting (material.rs:38-82)
__device__ __forceinline__ V3 lighting(const ShadeRec& m, cLightRec L, V3 point, V3 eyev, V3 normal,
                                       bool in_shadow) {
  const V3 color = m.pattern_kind >= 0 ? pattern_color(m, point)
                                       : v3(m.color[0], m.color[1], m.color[2]);
  const V3 intensity = v3(L->intensity[0], L->intensity[1], L->intensity[2]);
  const V3 effective_color = vmul(color, intensity);
  const V3 lightv = vnormalize(vsub(v3(L->pos[0], L->pos[1], L->pos[2]), point));
  const V3 ambient = vscale(effective_color, m.ambient);
  if (in_shadow) return ambient;
  const double light_dot_normal = vdot(lightv, normal);
  V3 diffuse = v3(0.0, 0.0, 0.0), specular = v3(0.0, 0.0, 0.0);
  if (!(light_dot_normal < 0.0)) {
    diffuse = vscale(vscale(effective_color, m.diffuse), light_dot_normal);
    const V3 reflectv = vreflect(vneg(lightv), normal);
    const double reflect_dot_eye = vdot(reflectv, eyev);
    if (!(reflect_dot_eye <= 0.0)) {
      const double factor = pow(reflect_dot_eye, m.shininess);
      specular = vscale(vscale(intensity, m.specular), factor);
    }
  }
  return vadd(vadd(ambient, diffuse), specular);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// camera.rs:57-69
__device__ __forceinline__ void ray_for_pixel(const DevCamera& cam, uint32_t px, uint32_t py, V3& o,
                                              V3& d) {
  const double xoffset = ((double)px + 0.5) * cam.pixel_size;
  const double yoffset = ((double)py + 0.5) * cam.pixel_size;
  const double world_x = cam.half_width - xoffset;
  const double world_y = cam.half_height - yoffset;
  const V3 pixel = m34_point(cam.inv, v3(world_x, world_y, -1.0));
  o = m34_point(cam.inv, v3(0.0, 0.0, 0.0));
  d = vnormalize(vsub(pixel, o));
}

}  // namespace rtamd
