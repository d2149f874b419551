// rt_device.hpp — device-side building blocks of the render path, shared by
// the wavefront pipeline (rt_wavefront.hip) and the batch kernels
// (rt_kernels.hip). Every function restates a reference function (cited),
// in binary64 with the reference's operation order; include only from .hip
// files compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rt_layout.hpp"
#include "rt_pow.hpp"

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
typedef const RT_CONST QuadRec* cQuadRec;
typedef const RT_CONST GroupRec* cGroupRec;
typedef const RT_CONST ConeCluster* cConeCluster;
typedef const RT_CONST LightRec* cLightRec;

typedef double d2 __attribute__((ext_vector_type(2)));  // ds_read_b128 operand
__host__ __device__ constexpr size_t lds_align16(size_t x) { return (x + 15) & ~(size_t)15; }

// ------------------------------------------------------------ trace (hot loop)
// World::intersect + intersections + hit (world.rs:31-38, intersection.rs:
// 108-125) without building or sorting the list: the nearest t >= 0 by
// (t, key) is the element the stable sort puts first, and the `containers`
// walk of prepare_computations (intersection.rs:63-90) only ever needs the two
// most recently entered containers (DESIGN.md "containers walk -> top-2").
struct Hit {
  double t;   // nearest t >= 0 (over eligible objects)
  int key;    // (object << kKeyShift) | list position, -1 = miss
  int hin;    // the hit object is in `containers` when the hit is reached
  // containers candidates (radiance rays): objects with an odd number of
  // intersections t < 0, keyed by their last such intersection; top 2.
  double c1t, c2t;
  int c1k, c2k;
};

__device__ __forceinline__ void hit_init(Hit& h) {
  h.t = INFINITY;
  h.key = 0x7fffffff;
  h.hin = 0;
  h.c1t = -INFINITY; h.c2t = -INFINITY; h.c1k = -1; h.c2k = -1;
}
__device__ __forceinline__ void hit_finish(Hit& h) {
  if (h.key == 0x7fffffff) h.key = -1;
}
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

// Sphere::local_intersect (sphere.rs:47-62) from (a, dt = d.o, c) of the
// object-space ray. With b = 2*dt and disc = b*b - (4a)*c = 4*(dt*dt - a*c)
// exactly (power-of-two scaling commutes with rounding), t = (-b -/+
// sqrt(disc)) / (2a) equals (-dt -/+ sqrt(dt*dt - a*c)) / a bit for bit
// (DESIGN.md "Sphere roots"). The object index / shadow flag (`meta`) is read
// only when disc >= 0. Root 1 can only be the hit when root 0 < 0, i.e. when
// the sphere is a container at the hit.
template <bool SHADOW, typename MetaFn>
__device__ __forceinline__ void sphere_adc(double a, double dt, double c, MetaFn meta_fn, Hit& h,
                                           unsigned& n_disc) {
  const double disc = dt * dt - a * c;
  if (disc >= 0.0) {
    ++n_disc;
    const int meta = meta_fn();
    const double q = sqrt(disc);
    const double t1 = (-dt - q) / a;
    const int k1 = (meta >> 1) << kKeyShift;
    const bool eligible = !SHADOW || (meta & 1);
    if (t1 >= 0.0) {
      if (eligible && better(t1, k1, h.t, h.key)) { h.t = t1; h.key = k1; h.hin = 0; }
    } else {  // root 2 matters only now (t1 < 0 or NaN): its division is left out otherwise
      const double t2 = (-dt + q) / a;
      if (eligible && t2 >= 0.0 && better(t2, k1 + 1, h.t, h.key)) { h.t = t2; h.key = k1 + 1; h.hin = 1; }
      if (!SHADOW && t1 < 0.0 && t2 >= 0.0) push_container(h, t1, k1);
    }
  }
}
template <bool SHADOW, typename MetaFn>
__device__ __forceinline__ void sphere_test(double ox, double oy, double oz, double dx, double dy, double dz,
                                            MetaFn meta_fn, Hit& h, unsigned& n_disc) {
  const double a = dx * dx + dy * dy + dz * dz;
  const double dt = dx * ox + dy * oy + dz * oz;
  const double c = ox * ox + oy * oy + oz * oz - 1.0;
  sphere_adc<SHADOW>(a, dt, c, meta_fn, h, n_disc);
}

// Plane::local_intersect (plane.rs:53-60) from the object-space y of origin
// and direction.
template <bool SHADOW>
__device__ __forceinline__ void plane_test(double oy, double dy, int meta, Hit& h) {
  if (!(fabs(dy) < kEpsilon)) {
    // a shadow ray moving away from the plane (oy, dy of one sign, the quotient far
    // from underflow): t < 0, no blocker, and its division is left out (the
    // closest hit needs t < 0 for `containers`)
    if (SHADOW && (oy > 0.0) == (dy > 0.0) && fabs(oy) > 1e-280 && fabs(dy) < 1e20) return;
    const double t = -oy / dy;
    const int k = (meta >> 1) << kKeyShift;
    const bool eligible = !SHADOW || (meta & 1);
    if (eligible && t >= 0.0 && better(t, k, h.t, h.key)) { h.t = t; h.key = k; h.hin = 0; }
    if (!SHADOW && t < 0.0) push_container(h, t, k);
  }
}

// Cube::check_axis (cube.rs:30-47)
__device__ __forceinline__ void cube_check_axis(double origin, double direction, double& tmin, double& tmax) {
  const double tmin_numerator = -1.0 - origin;
  const double tmax_numerator = 1.0 - origin;
  if (fabs(direction) >= kEpsilon) {
    tmin = tmin_numerator / direction;
    tmax = tmax_numerator / direction;
  } else {
    tmin = tmin_numerator * INFINITY;
    tmax = tmax_numerator * INFINITY;
  }
  if (tmin > tmax) { const double x = tmin; tmin = tmax; tmax = x; }
}
// Cylinder::check_cap (cylinder.rs:42-46, radius 1) / Cone::check_cap
// (cone.rs:67-71, radius = the cap's y)
__device__ __forceinline__ bool check_cap(V3 o, V3 d, double t, double radius) {
  const double x = o.x + t * d.x;
  const double z = o.z + t * d.z;
  return (x * x + z * z) <= radius * radius;
}
// intersect_caps (cylinder.rs:48-65, cone.rs:48-65): appends to t[n..]
__device__ __forceinline__ int intersect_caps(int kind, double mn, double mx, bool closed, V3 o, V3 d, double* t,
                                              int n) {
  if (!closed) return n;
  const bool cone = kind == 4;
  double tc = (mn - o.y) / d.y;
  if (check_cap(o, d, tc, cone ? mn : 1.0)) t[n++] = tc;
  tc = (mx - o.y) / d.y;
  if (check_cap(o, d, tc, cone ? mx : 1.0)) t[n++] = tc;
  return n;
}
// Cube / Cylinder / Cone local_intersect (cube.rs:71-93, cylinder.rs:88-119,
// cone.rs:94-134): the reference's list, in push order, into t[0..n).
__device__ __forceinline__ int quad_local_intersect(int kind, double mn, double mx, bool closed, V3 o, V3 d,
                                                    double t[4]) {
  if (kind == 2) {
    double xtmin, xtmax, ytmin, ytmax, ztmin, ztmax;
    cube_check_axis(o.x, d.x, xtmin, xtmax);
    cube_check_axis(o.y, d.y, ytmin, ytmax);
    cube_check_axis(o.z, d.z, ztmin, ztmax);
    const double tmin = fmax(fmax(xtmin, ytmin), ztmin);  // f64::max: NaN-ignoring
    const double tmax = fmin(fmin(xtmax, ytmax), ztmax);
    if (tmin > tmax) return 0;
    t[0] = tmin; t[1] = tmax;
    return 2;
  }
  double a, b, c;
  if (kind == 3) {
    a = d.x * d.x + d.z * d.z;
    if (fabs(a) < kEpsilon) return intersect_caps(kind, mn, mx, closed, o, d, t, 0);
    b = 2.0 * o.x * d.x + 2.0 * o.z * d.z;
    c = o.x * o.x + o.z * o.z - 1.0;
  } else {
    a = d.x * d.x - d.y * d.y + d.z * d.z;
    b = 2.0 * o.x * d.x - 2.0 * o.y * d.y + 2.0 * o.z * d.z;
    c = o.x * o.x - o.y * o.y + o.z * o.z;
    if (fabs(a) < kEpsilon) {
      if (fabs(b) < kEpsilon) return intersect_caps(kind, mn, mx, closed, o, d, t, 0);
      t[0] = -c / 2.0 * b;  // sic (cone.rs:104)
      return intersect_caps(kind, mn, mx, closed, o, d, t, 1);
    }
  }
  const double disc = b * b - 4.0 * a * c;
  if (disc < 0.0) return 0;  // no caps either (cylinder.rs:103-105, cone.rs:113-115)
  const double q = sqrt(disc);
  const double t0 = (-b - q) / (2.0 * a);
  const double t1 = (-b + q) / (2.0 * a);
  int n = 0;
  const double y0 = o.y + t0 * d.y;
  if (mn < y0 && y0 < mx) t[n++] = t0;
  const double y1 = o.y + t1 * d.y;
  if (mn < y1 && y1 < mx) t[n++] = t1;
  return intersect_caps(kind, mn, mx, closed, o, d, t, n);
}
// Shape::intersect (geometry/mod.rs:46-49) of one QuadRec, folded into `h`:
// the nearest t >= 0 of the object's list competes by (t, key); an object
// with an odd number of t < 0 is a container, ordered by its last one.
template <bool SHADOW, typename QP>  // QP: constant-address (wave-uniform) or generic record pointer
__device__ __forceinline__ void quad_test(QP q, V3 o, V3 d, Hit& h) {
  const V3 lo = v3(q->m[0] * o.x + q->m[1] * o.y + q->m[2] * o.z + q->m[3],
                   q->m[4] * o.x + q->m[5] * o.y + q->m[6] * o.z + q->m[7],
                   q->m[8] * o.x + q->m[9] * o.y + q->m[10] * o.z + q->m[11]);
  const V3 ld = v3(q->m[0] * d.x + q->m[1] * d.y + q->m[2] * d.z, q->m[4] * d.x + q->m[5] * d.y + q->m[6] * d.z,
                   q->m[8] * d.x + q->m[9] * d.y + q->m[10] * d.z);
  double t[4];
  const int n = quad_local_intersect(q->kind, q->minimum, q->maximum, q->closed != 0, lo, ld, t);
  if (n == 0) return;
  const int meta = q->meta;
  const int k0 = (meta >> 1) << kKeyShift;
  int n_neg = 0, neg_i = -1, best_i = -1;
  double neg_t = -INFINITY, best_t = INFINITY;
  for (int i = 0; i < n; ++i) {
    if (t[i] < 0.0) {
      ++n_neg;
      if (t[i] >= neg_t) { neg_t = t[i]; neg_i = i; }
    } else if (t[i] >= 0.0 && t[i] < best_t) {
      best_t = t[i]; best_i = i;
    }
  }
  const bool eligible = !SHADOW || (meta & 1);
  if (eligible && best_i >= 0 && better(best_t, k0 + best_i, h.t, h.key)) {
    h.t = best_t; h.key = k0 + best_i; h.hin = n_neg & 1;
  }
  if (!SHADOW && (n_neg & 1)) push_container(h, neg_t, k0 + neg_i);
}

// BoundingBox::intersects (bounding_box.rs:95-136) of a Group's box, with the
// reference's operations: per axis (min - o) / d and (max - o) / d, or, when
// |d| < EPSILON, the numerators times infinity (0 * inf = NaN), swapped when
// reversed; then f64::max / f64::min, which ignore a NaN operand (fmax / fmin).
__device__ __forceinline__ void bbox_check_axis(double origin, double direction, double mn, double mx, double& t0,
                                                double& t1) {
  const double tmin_numerator = mn - origin, tmax_numerator = mx - origin;
  double tmin, tmax;
  if (fabs(direction) >= kEpsilon) {
    tmin = tmin_numerator / direction;
    tmax = tmax_numerator / direction;
  } else {
    tmin = tmin_numerator * INFINITY;
    tmax = tmax_numerator * INFINITY;
  }
  if (tmin > tmax) { t0 = tmax; t1 = tmin; } else { t0 = tmin; t1 = tmax; }
}
__device__ __forceinline__ bool bbox_intersects(cGroupRec g, V3 o, V3 d) {
  double x0, x1, y0, y1, z0, z1;
  bbox_check_axis(o.x, d.x, g->lo[0], g->hi[0], x0, x1);
  bbox_check_axis(o.y, d.y, g->lo[1], g->hi[1], y0, y1);
  bbox_check_axis(o.z, d.z, g->lo[2], g->hi[2], z0, z1);
  const double tmin = fmax(fmax(x0, y0), z0), tmax = fmin(fmin(x1, y1), z1);
  return tmin <= tmax;
}
// Group::intersect (group.rs:49-58): a shape inside groups is intersected only
// when the ray meets the box of every group around it, innermost first (the
// reference tests them outermost first and stops at the first miss; either
// order gives the same answer). `gate` = the record's gate (0: no group).
// A shape that fails it adds no intersection and no local_intersect call.
__device__ __forceinline__ bool group_gate(const DevScene& sc, int gate, V3 o, V3 d) {
  const cGroupRec groups = (cGroupRec)sc.groups;
  for (int g = gate; g > 0; g = groups[g - 1].parent)
    if (!bbox_intersects(groups + (g - 1), o, d)) return false;
  return true;
}
// Shapes a group's box kept out of a ray's World::intersect, by kind (the
// counted launches subtract them from the reference's rays x shapes).
struct GateSkips {
  unsigned sph = 0, plane = 0, other = 0;
};

// The records outside the sphere BVH (general-transform spheres, planes,
// cubes / cylinders / cones), tested exhaustively from global memory.
// QUADS = false compiles the solids out (kernel variants for scenes without
// them keep the sphere loops' register allocation, hence their occupancy).
// FAST: the fast path's remainder (the records outside both hierarchies;
// the other bounded records are traversed by other_trace).
template <bool SHADOW, bool QUADS = true, bool FAST = false>
__device__ __forceinline__ void trace_rest(const DevScene& sc, V3 o, V3 d, Hit& h, unsigned& n_disc,
                                           GateSkips* skips = nullptr) {
  cSphereGen sg = (cSphereGen)(FAST ? sc.fx_gen : sc.sph_gen);
  const int n_gen = FAST ? sc.n_fx_gen : sc.n_gen;
  for (int j = 0; j < n_gen; ++j) {
    if (sg[j].gate && !group_gate(sc, sg[j].gate, o, d)) {
      if (skips) ++skips->sph;
      continue;
    }
    double m[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) m[e] = sg[j].m[e];
    const V3 lo = m34_point(m, o);
    const V3 ld = v3(m[0] * d.x + m[1] * d.y + m[2] * d.z, m[4] * d.x + m[5] * d.y + m[6] * d.z,
                     m[8] * d.x + m[9] * d.y + m[10] * d.z);
    sphere_test<SHADOW>(lo.x, lo.y, lo.z, ld.x, ld.y, ld.z, [&] { return (int)sg[j].meta; }, h, n_disc);
  }
  cPlaneRec pl = (cPlaneRec)sc.planes;
  for (int j = 0; j < sc.n_planes; ++j) {
    if (pl[j].gate && !group_gate(sc, pl[j].gate, o, d)) {
      if (skips) ++skips->plane;
      continue;
    }
    const double oy = pl[j].m[0] * o.x + pl[j].m[1] * o.y + pl[j].m[2] * o.z + pl[j].m[3];
    const double dy = pl[j].m[0] * d.x + pl[j].m[1] * d.y + pl[j].m[2] * d.z;
    plane_test<SHADOW>(oy, dy, (int)pl[j].meta, h);
  }
  if constexpr (QUADS) {
    cQuadRec qr = (cQuadRec)(FAST ? sc.fx_quads : sc.quads);
    const int n_quads = FAST ? sc.n_fx_quads : sc.n_quads;
    for (int j = 0; j < n_quads; ++j) {
      if (qr[j].gate && !group_gate(sc, qr[j].gate, o, d)) {
        if (skips) ++skips->other;
        continue;
      }
      quad_test<SHADOW>(qr + j, o, d, h);
    }
  }
}

// One culled other record (rt_layout.hpp OtherRec) with exactly the
// operations of the exhaustive loops above: a general sphere as trace_rest's
// general records, a solid as quad_test; a record inside groups only when the
// ray meets every group box around it (group_gate, as trace_rest).
template <bool SHADOW>
__device__ __forceinline__ void other_test(const DevScene& sc, const OtherRec* q, V3 o, V3 d, Hit& h,
                                           unsigned& n_disc) {
  if (q->gate && !group_gate(sc, q->gate, o, d)) return;  // Group::intersect (group.rs:49-58)
  if (q->kind == 0) {
    const double* m = q->m;
    const V3 lo = m34_point(m, o);
    const V3 ld = v3(m[0] * d.x + m[1] * d.y + m[2] * d.z, m[4] * d.x + m[5] * d.y + m[6] * d.z,
                     m[8] * d.x + m[9] * d.y + m[10] * d.z);
    sphere_test<SHADOW>(lo.x, lo.y, lo.z, ld.x, ld.y, ld.z, [&] { return (int)q->meta; }, h, n_disc);
  } else {
    quad_test<SHADOW>(q, o, d, h);
  }
}

// One diagonal-inverse sphere record (global memory, scalar loads).
template <bool SHADOW>
__device__ __forceinline__ void diag_test(cSphereDiag r, V3 o, V3 d, Hit& h, unsigned& n_disc) {
  // off-diagonal inverse entries are exact zeros: ((m00*x + 0) + 0) + m03 == m00*x + m03
  const double s0 = r->s[0], s1 = r->s[1], s2 = r->s[2];
  sphere_test<SHADOW>(s0 * o.x + r->t[0], s1 * o.y + r->t[1], s2 * o.z + r->t[2], s0 * d.x, s1 * d.y, s2 * d.z,
                      [&] { return (int)r->meta; }, h, n_disc);
}

// Generic exhaustive trace over the scene's records in global memory (scalar
// loads): the batch entry points (rt_hit_batch, rt_is_shadowed_batch) and
// the wavefront fallback when the trace image does not fit in LDS.
template <bool SHADOW>
__device__ __forceinline__ void trace(const DevScene& sc, V3 o, V3 d, Hit& h, unsigned& n_disc,
                                      GateSkips* skips = nullptr) {
  hit_init(h);
  cSphereDiag sd = (cSphereDiag)sc.sph_diag;
  for (int j = 0; j < sc.n_diag; ++j) diag_test<SHADOW>(sd + j, o, d, h, n_disc);
  trace_rest<SHADOW>(sc, o, d, h, n_disc, skips);
  hit_finish(h);
}

// --------------------------------------------------------------- shading
struct Comps {
  V3 point, over, under, eyev, normal;
  double n1, n2;
  int obj;
  bool inside;
};

// Shape::local_normal_at per kind (sphere.rs:64-67, plane.rs:62-64,
// cube.rs:95-106, cylinder.rs:121-130, cone.rs:136-149).
__device__ __forceinline__ V3 local_normal_at(const ShadeRec& s, V3 p) {
  switch (s.kind) {
    case 0: return vsub(p, v3(0.0, 0.0, 0.0));
    case 1: return v3(0.0, 1.0, 0.0);
    case 2: {
      const double maxc = fmax(fmax(fabs(p.x), fabs(p.y)), fabs(p.z));
      if (req(maxc, fabs(p.x))) return v3(p.x, 0.0, 0.0);
      if (req(maxc, fabs(p.y))) return v3(0.0, p.y, 0.0);
      return v3(0.0, 0.0, p.z);
    }
    default: {
      const double dist = p.x * p.x + p.z * p.z;
      if (dist < 1.0 && p.y >= s.maximum - kEpsilon) return v3(0.0, 1.0, 0.0);
      if (dist < 1.0 && p.y <= s.minimum + kEpsilon) return v3(0.0, -1.0, 0.0);
      if (s.kind == 3) return v3(p.x, 0.0, p.z);
      double y = sqrt(p.x * p.x + p.z * p.z);
      if (p.y > 0.0) y = -y;
      return v3(p.x, y, p.z);
    }
  }
}

// Intersection::prepare_computations (intersection.rs:53-105) with the exact
// top-2 replacement of the containers walk.
__device__ __forceinline__ Comps prepare(const DevScene& sc, V3 o, V3 d, const Hit& h) {
  Comps c;
  const int obj = h.key >> kKeyShift;
  const ShadeRec& s = sc.shade[obj];
  c.obj = obj;
  c.point = vadd(o, vscale(d, h.t));  // ray.rs:22-24
  c.eyev = vneg(d);
  // Shape::normal_at (geometry/mod.rs:51-56)
  const V3 lp = m34_point(s.inv, c.point);
  V3 n = vnormalize(m33_vector(s.invT, local_normal_at(s, lp)));
  c.inside = false;
  if (vdot(n, c.eyev) < 0.0) { c.inside = true; n = vneg(n); }
  c.normal = n;
  // n1 / n2 (intersection.rs:63-90, DESIGN.md "containers walk -> top-2"):
  // n1 = last container before the hit; n2 = last after toggling the hit object
  c.n1 = h.c1k >= 0 ? sc.shade[h.c1k >> kKeyShift].refractive_index : 1.0;
  if (!h.hin) {
    c.n2 = s.refractive_index;
  } else if ((h.c1k >> kKeyShift) == obj) {
    c.n2 = h.c2k >= 0 ? sc.shade[h.c2k >> kKeyShift].refractive_index : 1.0;
  } else {
    c.n2 = sc.shade[h.c1k >> kKeyShift].refractive_index;
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

// `v % 2.0 == 0.0` (Rust's f64 `%` is fmod) for an integer-valued or
// non-finite v, without the fmod loop: binary64 values of magnitude >= 2^53
// are even integers, below that the integer conversion is exact.
__device__ __forceinline__ bool fmod2_is_zero(double v) {
  if (!(fabs(v) < 0x1p53)) return !isnan(v) && !isinf(v);
  return (((long long)v) & 1) == 0;
}

// componentwise select (a select between whole structs becomes a scratch
// copy indexed by the condition)
__device__ __forceinline__ V3 vsel(bool c, V3 a, V3 b) { return v3(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z); }

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
      return vsel(fmod2_is_zero(floor(pp.x)), a, b);
    case 2: {  // gradient.rs:14-18
      const V3 distance = vsub(b, a);
      const double fraction = pp.x - floor(pp.x);
      return vadd(a, vscale(distance, fraction));
    }
    case 3: {  // ring.rs:14-21
      const double distance = floor(sqrt(pp.x * pp.x + pp.z * pp.z));
      return vsel(fmod2_is_zero(distance), a, b);
    }
    default: {  // checkers.rs:14-21: `as isize` (saturating) then % 2
      const double distance = floor(pp.x) + floor(pp.y) + floor(pp.z);
      bool even;
      if (isnan(distance)) even = true;                          // NaN as isize = 0
      else if (distance >= 9223372036854775808.0) even = false;  // isize::MAX is odd
      else if (distance < -9223372036854775808.0) even = true;   // isize::MIN is even
      else even = fmod2_is_zero(distance);                      // exact integer parity
      return vsel(even, a, b);
    }
  }
}

// f64::powf of the specular term (material.rs:76): glibc 2.35's pow, operation
// for operation (rt_pow.hpp), so the colours are the reference host's bit for
// bit (OCML's pow differed by 1-2 ulps in about 1 of 4000 channels, round 5);
// the frame costs the same (profiles/r06_ab_pow.txt: +0.2 %, within noise).
// Out of line: inlined into the fused trace kernels, its constants were hoisted
// out of the ray loop into VGPRs and spilled across the BVH traversal.
__device__ __attribute__((noinline)) double spec_pow(double x, double y) { return pow_glibc(x, y); }

// Material::lighting (material.rs:38-82)
// `lightv` = (light.position - point).normalize(), which the caller may
// already hold: the shadow ray from `point` to the light has exactly that
// direction (same operands, same operations), so the shadow trace passes it.
__device__ __forceinline__ V3 lighting(const ShadeRec& m, cLightRec L, V3 point, V3 eyev, V3 normal,
                                       bool in_shadow, V3 lightv) {
  const V3 color = m.pattern_kind >= 0 ? pattern_color(m, point)
                                       : v3(m.color[0], m.color[1], m.color[2]);
  const V3 intensity = v3(L->intensity[0], L->intensity[1], L->intensity[2]);
  const V3 effective_color = vmul(color, intensity);
  const V3 ambient = vscale(effective_color, m.ambient);
  if (in_shadow) return ambient;
  const double light_dot_normal = vdot(lightv, normal);
  V3 diffuse = v3(0.0, 0.0, 0.0), specular = v3(0.0, 0.0, 0.0);
  if (!(light_dot_normal < 0.0)) {
    diffuse = vscale(vscale(effective_color, m.diffuse), light_dot_normal);
    const V3 reflectv = vreflect(vneg(lightv), normal);
    const double reflect_dot_eye = vdot(reflectv, eyev);
    if (!(reflect_dot_eye <= 0.0)) {
      // A material without specular (e.g. the C3/C5 floors): (I * 0) * f equals
      // I * 0 bit for bit whenever f = pow(x, y) is finite and not -0, which holds
      // for 0 < x <= 1 and 0 <= y < inf (f in [0, 1]); then pow need not run.
      const bool no_spec = m.specular == 0.0 && reflect_dot_eye <= 1.0 && m.shininess >= 0.0 &&
                           m.shininess < INFINITY && fabs(intensity.x) < INFINITY &&
                           fabs(intensity.y) < INFINITY && fabs(intensity.z) < INFINITY;
      if (no_spec) {
        specular = vscale(intensity, m.specular);
      } else {
        const double factor = spec_pow(reflect_dot_eye, m.shininess);
        specular = vscale(vscale(intensity, m.specular), factor);
      }
    }
  }
  return vadd(vadd(ambient, diffuse), specular);
}
__device__ __forceinline__ V3 lighting(const ShadeRec& m, cLightRec L, V3 point, V3 eyev, V3 normal,
                                       bool in_shadow) {
  return lighting(m, L, point, eyev, normal, in_shadow,
                  vnormalize(vsub(v3(L->pos[0], L->pos[1], L->pos[2]), point)));
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// camera.rs:57-69 (offsets 0.5, 0.5) and rays_for_pixel (camera.rs:71-90)
// with the AA sample offsets of get_offsets (camera.rs:92-126).
__device__ __forceinline__ void ray_for_pixel(const DevCamera& cam, uint32_t px, uint32_t py, V3& o, V3& d,
                                              double offx = 0.5, double offy = 0.5) {
  const double xoffset = ((double)px + offx) * cam.pixel_size;
  const double yoffset = ((double)py + offy) * cam.pixel_size;
  const double world_x = cam.half_width - xoffset;
  const double world_y = cam.half_height - yoffset;
  const V3 pixel = m34_point(cam.inv, v3(world_x, world_y, -1.0));
  o = m34_point(cam.inv, v3(0.0, 0.0, 0.0));
  d = vnormalize(vsub(pixel, o));
}

}  // namespace rtamd
