/*
 * rt_oracle.c — CPU parity ORACLE (test infrastructure only; see rt_oracle.h).
 *
 * Plain-C restatement of tlinford/raytracer-challenge-rs's render path. Every
 * function names the reference file:line it follows. Operation order is the
 * reference's (left-associative Rust expressions, no FMA: built with
 * -ffp-contract=off). Intersections are sorted with a STABLE sort so that
 * exact-t ties resolve in insertion order (object order, t1 before t2): the
 * reference's `sort_unstable_by` (geometry/intersection.rs:113) is an
 * insertion sort for short lists, which is stable; for long lists exact ties
 * are measure-zero (DESIGN.md "Tie order").
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread int g_nan_seen = 0;
int oracle_nan_seen(void) { return g_nan_seen; }

/* ---------------------------------------------------------------- lib.rs */
/* lib.rs:20-22 */
int or_equal(double a, double b) { return fabs(a - b) < OR_EPSILON; }

/* lib.rs:24-31 (including its sign-test quirk) */
static int or_equal_ignore_inf(double a, double b) {
  if (isinf(a) && isinf(b)) {
    return (!signbit(a) && !signbit(a)) || (signbit(b) && signbit(b));
  }
  return or_equal(a, b);
}

/* ------------------------------------------- vector.rs / point.rs / color.rs */
ot3 or_t3(double x, double y, double z) { ot3 r = {x, y, z}; return r; }
ot3 or_add(ot3 a, ot3 b) { return or_t3(a.x + b.x, a.y + b.y, a.z + b.z); }
ot3 or_sub(ot3 a, ot3 b) { return or_t3(a.x - b.x, a.y - b.y, a.z - b.z); }
ot3 or_neg(ot3 a) { return or_t3(-a.x, -a.y, -a.z); }
ot3 or_scale(ot3 a, double s) { return or_t3(a.x * s, a.y * s, a.z * s); }
ot3 or_hadamard(ot3 a, ot3 b) { return or_t3(a.x * b.x, a.y * b.y, a.z * b.z); }
/* vector.rs:99-101 */
double or_dot(ot3 a, ot3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* vector.rs:103-109 */
ot3 or_cross(ot3 a, ot3 b) {
  return or_t3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* vector.rs:21-23 */
double or_magnitude(ot3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
/* vector.rs:25-28 */
ot3 or_normalize(ot3 a) {
  double m = or_magnitude(a);
  return or_t3(a.x / m, a.y / m, a.z / m);
}
/* vector.rs:30-32: self - normal * 2.0 * dot(self, normal) */
ot3 or_reflect(ot3 v, ot3 n) { return or_sub(v, or_scale(or_scale(n, 2.0), or_dot(v, n))); }
/* vector.rs:35-41 / point.rs:32-36 / color.rs:36-42 */
int or_t3_eq(ot3 a, ot3 b) { return or_equal(a.x, b.x) && or_equal(a.y, b.y) && or_equal(a.z, b.z); }
/* point.rs:26-30 */
static int or_t3_eq_ignore_inf(ot3 a, ot3 b) {
  return or_equal_ignore_inf(a.x, b.x) && or_equal_ignore_inf(a.y, b.y) &&
         or_equal_ignore_inf(a.z, b.z);
}

/* -------------------------------------------------------------- matrix.rs */
omat om_zero(int r, int c) { omat m; memset(&m, 0, sizeof m); m.rows = r; m.cols = c; return m; }
/* matrix.rs:28-36 */
omat om_identity(int n) { omat m = om_zero(n, n); for (int i = 0; i < n; ++i) m.e[i * n + i] = 1.0; return m; }
omat om_from(int r, int c, const double* e) { omat m = om_zero(r, c); memcpy(m.e, e, sizeof(double) * r * c); return m; }
/* matrix.rs:75-77 */
double om_at(const omat* m, int i, int j) { return m->e[i * m->cols + j]; }
static void om_set(omat* m, int i, int j, double v) { m->e[i * m->cols + j] = v; }

/* matrix.rs:210-230 */
omat om_mul(const omat* a, const omat* b) {
  omat m = om_zero(a->rows, b->cols);
  for (int row = 0; row < a->rows; ++row)
    for (int col = 0; col < b->cols; ++col) {
      double c = 0.0;
      for (int i = 0; i < a->cols; ++i) c += om_at(a, row, i) * om_at(b, i, col);
      om_set(&m, row, col, c);
    }
  return m;
}
/* matrix.rs:232-245 (row 3 ignored) */
ot3 om_mul_point(const omat* m, ot3 p) {
  return or_t3(om_at(m, 0, 0) * p.x + om_at(m, 0, 1) * p.y + om_at(m, 0, 2) * p.z + om_at(m, 0, 3),
               om_at(m, 1, 0) * p.x + om_at(m, 1, 1) * p.y + om_at(m, 1, 2) * p.z + om_at(m, 1, 3),
               om_at(m, 2, 0) * p.x + om_at(m, 2, 1) * p.y + om_at(m, 2, 2) * p.z + om_at(m, 2, 3));
}
/* matrix.rs:247-260 */
ot3 om_mul_vector(const omat* m, ot3 v) {
  return or_t3(om_at(m, 0, 0) * v.x + om_at(m, 0, 1) * v.y + om_at(m, 0, 2) * v.z,
               om_at(m, 1, 0) * v.x + om_at(m, 1, 1) * v.y + om_at(m, 1, 2) * v.z,
               om_at(m, 2, 0) * v.x + om_at(m, 2, 1) * v.y + om_at(m, 2, 2) * v.z);
}
/* matrix.rs:79-89 */
omat om_transpose(const omat* m) {
  omat t = om_zero(m->cols, m->rows);
  for (int i = 0; i < m->rows; ++i)
    for (int j = 0; j < m->cols; ++j) om_set(&t, j, i, om_at(m, i, j));
  return t;
}
/* matrix.rs:91-102 */
double om_determinant(const omat* m) {
  if (m->rows == 2 && m->cols == 2) return om_at(m, 0, 0) * om_at(m, 1, 1) - om_at(m, 0, 1) * om_at(m, 1, 0);
  double det = 0.0;
  for (int col = 0; col < m->cols; ++col) det += om_at(m, 0, col) * om_cofactor(m, 0, col);
  return det;
}
/* matrix.rs:104-120 */
omat om_submatrix(const omat* m, int row, int col) {
  omat s = om_zero(m->rows - 1, m->cols - 1);
  for (int i = 0; i < s.rows; ++i)
    for (int j = 0; j < s.cols; ++j) {
      int ii = i < row ? i : i + 1, jj = j < col ? j : j + 1;
      om_set(&s, i, j, om_at(m, ii, jj));
    }
  return s;
}
/* matrix.rs:122-124 */
double om_minor(const omat* m, int row, int col) { omat s = om_submatrix(m, row, col); return om_determinant(&s); }
/* matrix.rs:126-132 */
double om_cofactor(const omat* m, int row, int col) {
  return ((row + col) % 2 == 1) ? -om_minor(m, row, col) : om_minor(m, row, col);
}
/* matrix.rs:134-136 */
int om_is_invertible(const omat* m) { return !or_equal(om_determinant(m), 0.0); }
/* matrix.rs:138-153: inv[j][i] = cofactor(i,j) / det */
int om_inverse(const omat* m, omat* out) {
  if (!om_is_invertible(m) || m->rows != m->cols) return RT_ERR_NOT_INVERTIBLE;
  omat inv = om_zero(m->rows, m->cols);
  double det = om_determinant(m);
  for (int i = 0; i < m->rows; ++i)
    for (int j = 0; j < m->cols; ++j) om_set(&inv, j, i, om_cofactor(m, i, j) / det);
  *out = inv;
  return RT_OK;
}
/* matrix.rs:201-208 */
int om_eq(const omat* a, const omat* b) {
  int n = a->rows * a->cols, nb = b->rows * b->cols;
  if (nb < n) n = nb; /* zip stops at the shorter */
  for (int i = 0; i < n; ++i) if (!or_equal(a->e[i], b->e[i])) return 0;
  return 1;
}

/* ----------------------------------------------------------- transform.rs */
omat or_translation(double x, double y, double z) { /* :7-15 */
  omat t = om_identity(4); om_set(&t, 0, 3, x); om_set(&t, 1, 3, y); om_set(&t, 2, 3, z); return t;
}
omat or_scaling(double x, double y, double z) { /* :17-25 */
  omat s = om_identity(4); om_set(&s, 0, 0, x); om_set(&s, 1, 1, y); om_set(&s, 2, 2, z); return s;
}
omat or_rotation_x(double r) { /* :27-36 */
  omat m = om_identity(4);
  om_set(&m, 1, 1, cos(r)); om_set(&m, 1, 2, -sin(r)); om_set(&m, 2, 1, sin(r)); om_set(&m, 2, 2, cos(r));
  return m;
}
omat or_rotation_y(double r) { /* :38-47 */
  omat m = om_identity(4);
  om_set(&m, 0, 0, cos(r)); om_set(&m, 0, 2, sin(r)); om_set(&m, 2, 0, -sin(r)); om_set(&m, 2, 2, cos(r));
  return m;
}
omat or_rotation_z(double r) { /* :49-58 */
  omat m = om_identity(4);
  om_set(&m, 0, 0, cos(r)); om_set(&m, 0, 1, -sin(r)); om_set(&m, 1, 0, sin(r)); om_set(&m, 1, 1, cos(r));
  return m;
}
omat or_shearing(double xy, double xz, double yx, double yz, double zx, double zy) { /* :60-71 */
  omat s = om_identity(4);
  om_set(&s, 0, 1, xy); om_set(&s, 0, 2, xz); om_set(&s, 1, 0, yx);
  om_set(&s, 1, 2, yz); om_set(&s, 2, 0, zx); om_set(&s, 2, 1, zy);
  return s;
}
omat or_view_transform(ot3 from, ot3 to, ot3 up) { /* :73-90 */
  ot3 forward = or_normalize(or_sub(to, from));
  ot3 upn = or_normalize(up);
  ot3 left = or_cross(forward, upn);
  ot3 true_up = or_cross(left, forward);
  double e[16] = {left.x, left.y, left.z, 0.0,
                  true_up.x, true_up.y, true_up.z, 0.0,
                  -forward.x, -forward.y, -forward.z, 0.0,
                  0.0, 0.0, 0.0, 1.0};
  omat orientation = om_from(4, 4, e);
  omat tr = or_translation(-from.x, -from.y, -from.z);
  return om_mul(&orientation, &tr);
}

/* -------------------------------------------------------- bounding_box.rs */
static obbox or_bbox_default(void) { /* :12-19 */
  obbox b = {or_t3(INFINITY, INFINITY, INFINITY), or_t3(-INFINITY, -INFINITY, -INFINITY)};
  return b;
}
static void or_bbox_add_point(obbox* b, ot3 p) { /* :31-52 */
  if (p.x > b->max.x) b->max.x = p.x;
  if (p.y > b->max.y) b->max.y = p.y;
  if (p.z > b->max.z) b->max.z = p.z;
  if (p.x < b->min.x) b->min.x = p.x;
  if (p.y < b->min.y) b->min.y = p.y;
  if (p.z < b->min.z) b->min.z = p.z;
}
static obbox or_bbox_transform(const obbox* b, const omat* m) { /* :71-89 */
  ot3 pts[8] = {b->min,
                or_t3(b->min.x, b->min.y, b->max.z),
                or_t3(b->min.x, b->max.y, b->min.z),
                or_t3(b->min.x, b->max.y, b->max.z),
                or_t3(b->max.x, b->min.y, b->min.z),
                or_t3(b->max.x, b->min.y, b->max.z),
                or_t3(b->max.x, b->max.y, b->min.z),
                b->max};
  obbox nb = or_bbox_default();
  for (int i = 0; i < 8; ++i) or_bbox_add_point(&nb, om_mul_point(m, pts[i]));
  return nb;
}
static int or_bbox_eq(const obbox* a, const obbox* b) { /* :20-24 */
  return or_t3_eq_ignore_inf(a->min, b->min) && or_t3_eq_ignore_inf(a->max, b->max);
}
/* :118-136: per axis (min - o) / d and (max - o) / d, or the numerators times
 * infinity when |d| < EPSILON (0 * inf is NaN), ordered */
static void or_bbox_check_axis(double origin, double direction, double mn, double mx, double* t0, double* t1) {
  double tmin_numerator = mn - origin;
  double tmax_numerator = mx - origin;
  double tmin, tmax;
  if (fabs(direction) >= OR_EPSILON) {
    tmin = tmin_numerator / direction;
    tmax = tmax_numerator / direction;
  } else {
    tmin = tmin_numerator * INFINITY;
    tmax = tmax_numerator * INFINITY;
  }
  if (tmin > tmax) { *t0 = tmax; *t1 = tmin; } else { *t0 = tmin; *t1 = tmax; }
}
/* :95-116 (f64::max / f64::min ignore a NaN operand: fmax / fmin) */
int or_bbox_intersects(const obbox* b, const oray* r) {
  double x0, x1, y0, y1, z0, z1;
  or_bbox_check_axis(r->origin.x, r->direction.x, b->min.x, b->max.x, &x0, &x1);
  or_bbox_check_axis(r->origin.y, r->direction.y, b->min.y, b->max.y, &y0, &y1);
  or_bbox_check_axis(r->origin.z, r->direction.z, b->min.z, b->max.z, &z0, &z1);
  double tmin = fmax(fmax(x0, y0), z0);
  double tmax = fmin(fmin(x1, y1), z1);
  return tmin <= tmax;
}

/* -------------------------------------------------------- pattern/{mod,stripe,gradient,ring,checkers,test_pattern}.rs */
opattern or_pattern(int kind, ot3 a, ot3 b) { /* pattern/mod.rs:23-31,60-91 */
  opattern p;
  p.kind = kind; p.a = a; p.b = b;
  p.transform = om_identity(4); p.inverse = om_identity(4);
  return p;
}
void or_pattern_set_transform(opattern* p, const omat* t) { /* pattern/mod.rs:34-37 */
  p->transform = *t;
  om_inverse(t, &p->inverse);
}
static int or_pattern_eq(const opattern* a, const opattern* b) { /* derived PartialEq */
  return om_eq(&a->transform, &b->transform) && om_eq(&a->inverse, &b->inverse) &&
         a->kind == b->kind &&
         (a->kind == RT_PATTERN_TEST || (or_t3_eq(a->a, b->a) && or_t3_eq(a->b, b->b)));
}
ot3 or_pattern_color_at(const opattern* p, ot3 pt) {
  switch (p->kind) {
    case RT_PATTERN_TEST: /* test_pattern.rs:7-9 */
      return or_t3(pt.x, pt.y, pt.z);
    case RT_PATTERN_STRIPE: /* stripe.rs:14-20 */
      return fmod(floor(pt.x), 2.0) == 0.0 ? p->a : p->b;
    case RT_PATTERN_GRADIENT: { /* gradient.rs:14-18 */
      ot3 distance = or_sub(p->b, p->a);
      double fraction = pt.x - floor(pt.x);
      return or_add(p->a, or_scale(distance, fraction));
    }
    case RT_PATTERN_RING: { /* ring.rs:14-21 */
      double distance = floor(sqrt(pt.x * pt.x + pt.z * pt.z));
      return fmod(distance, 2.0) == 0.0 ? p->a : p->b;
    }
    case RT_PATTERN_CHECKERS: { /* checkers.rs:14-21; `as isize` saturates */
      double distance = floor(pt.x) + floor(pt.y) + floor(pt.z);
      long long d;
      if (isnan(distance)) d = 0;
      else if (distance >= 9223372036854775807.0) d = INT64_MAX;
      else if (distance <= -9223372036854775808.0) d = INT64_MIN;
      else d = (long long)distance;
      return (d % 2 == 0) ? p->a : p->b;
    }
  }
  return or_t3(0, 0, 0);
}
/* pattern/mod.rs:39-49 */
ot3 or_pattern_color_at_shape(const opattern* p, const oshape* s, ot3 world_point) {
  ot3 object_point = om_mul_point(&s->inverse, world_point);
  ot3 pattern_point = om_mul_point(&p->inverse, object_point);
  return or_pattern_color_at(p, pattern_point);
}

/* ------------------------------------------------------------ material.rs */
omaterial or_material_default(void) { /* :24-36 */
  omaterial m;
  memset(&m, 0, sizeof m);
  m.color = or_t3(1.0, 1.0, 1.0);
  m.ambient = 0.1; m.diffuse = 0.9; m.specular = 0.9; m.shininess = 200.0;
  m.reflective = 0.0; m.transparency = 0.0; m.refractive_index = 1.0;
  m.has_pattern = 0;
  return m;
}
static int or_material_eq(const omaterial* a, const omaterial* b) { /* derived PartialEq :10 */
  if (!or_t3_eq(a->color, b->color)) return 0;
  if (!(a->ambient == b->ambient && a->diffuse == b->diffuse && a->specular == b->specular &&
        a->shininess == b->shininess && a->reflective == b->reflective &&
        a->transparency == b->transparency && a->refractive_index == b->refractive_index))
    return 0;
  if (a->has_pattern != b->has_pattern) return 0;
  return !a->has_pattern || or_pattern_eq(&a->pattern, &b->pattern);
}

/* :38-82 */
ot3 or_lighting(const omaterial* m, const oshape* obj, const olight* light, ot3 point,
                ot3 eyev, ot3 normalv, int in_shadow) {
  ot3 color = m->has_pattern ? or_pattern_color_at_shape(&m->pattern, obj, point) : m->color;
  ot3 effective_color = or_hadamard(color, light->intensity);
  ot3 lightv = or_normalize(or_sub(light->position, point));
  ot3 ambient = or_scale(effective_color, m->ambient);
  if (in_shadow) return ambient;
  double light_dot_normal = or_dot(lightv, normalv);
  ot3 diffuse, specular;
  if (light_dot_normal < 0.0) {
    diffuse = or_t3(0.0, 0.0, 0.0);
    specular = or_t3(0.0, 0.0, 0.0);
  } else {
    diffuse = or_scale(or_scale(effective_color, m->diffuse), light_dot_normal);
    ot3 reflectv = or_reflect(or_neg(lightv), normalv);
    double reflect_dot_eye = or_dot(reflectv, eyev);
    if (reflect_dot_eye <= 0.0) {
      specular = or_t3(0.0, 0.0, 0.0);
    } else {
      double factor = pow(reflect_dot_eye, m->shininess);
      specular = or_scale(or_scale(light->intensity, m->specular), factor);
    }
  }
  return or_add(or_add(ambient, diffuse), specular);
}

/* ------------------------------------------------- geometry/mod.rs, shapes */
static oshape or_shape_base(int kind) { /* geometry/mod.rs:22-36 */
  oshape s;
  memset(&s, 0, sizeof s);
  s.kind = kind;
  s.transform = om_identity(4);
  s.inverse = om_identity(4);
  s.inverse_t = om_identity(4);
  s.material = or_material_default();
  s.bbox = or_bbox_default();
  s.shadow = 1;
  return s;
}
oshape or_sphere_default(void) { /* sphere.rs:16-25 */
  oshape s = or_shape_base(RT_SHAPE_SPHERE);
  s.bbox.min = or_t3(-1, -1, -1);
  s.bbox.max = or_t3(1, 1, 1);
  return s;
}
oshape or_sphere_glass(void) { /* sphere.rs:70-77 */
  oshape s = or_sphere_default();
  s.material.transparency = 1.0;
  s.material.refractive_index = 1.5;
  return s;
}
oshape or_plane_default(void) { /* plane.rs:19-31 */
  oshape s = or_shape_base(RT_SHAPE_PLANE);
  s.bbox.min = or_t3(-INFINITY, 0.0, -INFINITY);
  s.bbox.max = or_t3(INFINITY, 0.0, INFINITY);
  return s;
}
oshape or_cube_default(void) { /* cube.rs:17-26 */
  oshape s = or_shape_base(RT_SHAPE_CUBE);
  s.bbox.min = or_t3(-1, -1, -1);
  s.bbox.max = or_t3(1, 1, 1);
  return s;
}
oshape or_cylinder_new(double minimum, double maximum, int closed) { /* cylinder.rs:27-42 */
  oshape s = or_shape_base(RT_SHAPE_CYLINDER);
  s.bbox.min = or_t3(-1.0, minimum, -1.0);
  s.bbox.max = or_t3(1.0, maximum, 1.0);
  s.minimum = minimum; s.maximum = maximum; s.closed = closed ? 1 : 0;
  return s;
}
oshape or_cone_new(double minimum, double maximum, int closed) { /* cone.rs:26-47 */
  oshape s = or_shape_base(RT_SHAPE_CONE);
  double a = fabs(minimum), b = fabs(maximum);
  double limit = fmax(a, b); /* f64::max */
  s.bbox.min = or_t3(-limit, minimum, -limit);
  s.bbox.max = or_t3(limit, maximum, limit);
  s.minimum = minimum; s.maximum = maximum; s.closed = closed ? 1 : 0;
  return s;
}
/* geometry/mod.rs:74-85 */
int or_shape_set_transform(oshape* s, const omat* t) {
  s->bbox = or_bbox_transform(&s->bbox, &s->inverse);
  omat inv;
  int rc = om_inverse(t, &inv);
  if (rc != RT_OK) return rc;
  s->transform = *t;
  s->inverse = inv;
  s->inverse_t = om_transpose(&inv);
  s->bbox = or_bbox_transform(&s->bbox, &s->transform);
  return RT_OK;
}
/* sphere.rs:40-45 / plane.rs:46-51 / cube.rs:63-68 -> derived PartialEq of
 * BaseShape (mod.rs:12); Cylinder / Cone also compare minimum, maximum,
 * closed (derived PartialEq, cylinder.rs:12, cone.rs:12). */
int or_shape_equals(const oshape* a, const oshape* b) {
  if (a->kind != b->kind) return 0;
  if ((a->kind == RT_SHAPE_CYLINDER || a->kind == RT_SHAPE_CONE) &&
      !(a->minimum == b->minimum && a->maximum == b->maximum && a->closed == b->closed))
    return 0;
  return om_eq(&a->transform, &b->transform) && om_eq(&a->inverse, &b->inverse) &&
         om_eq(&a->inverse_t, &b->inverse_t) && or_material_eq(&a->material, &b->material) &&
         or_bbox_eq(&a->bbox, &b->bbox) && a->shadow == b->shadow;
}

/* cube.rs:29-47 */
static void or_cube_check_axis(double origin, double direction, double* tmin_out, double* tmax_out) {
  double tmin_numerator = -1.0 - origin;
  double tmax_numerator = 1.0 - origin;
  double tmin, tmax;
  if (fabs(direction) >= OR_EPSILON) {
    tmin = tmin_numerator / direction;
    tmax = tmax_numerator / direction;
  } else {
    tmin = tmin_numerator * INFINITY;
    tmax = tmax_numerator * INFINITY;
  }
  if (tmin > tmax) { double t = tmin; tmin = tmax; tmax = t; }
  *tmin_out = tmin; *tmax_out = tmax;
}
/* cylinder.rs:44-48 (radius 1) and cone.rs:70-74 (radius = the cap's y) */
static int or_check_cap(const oray* ray, double t, double radius) {
  double x = ray->origin.x + t * ray->direction.x;
  double z = ray->origin.z + t * ray->direction.z;
  return (x * x + z * z) <= radius * radius;
}
/* cylinder.rs:50-67 / cone.rs:52-68 */
static int or_intersect_caps(const oshape* s, const oray* ray, double* t_out, int n) {
  if (!s->closed) return n;
  int cone = s->kind == RT_SHAPE_CONE;
  double t = (s->minimum - ray->origin.y) / ray->direction.y;
  if (cone ? or_check_cap(ray, t, s->minimum) : or_check_cap(ray, t, 1.0)) t_out[n++] = t;
  t = (s->maximum - ray->origin.y) / ray->direction.y;
  if (cone ? or_check_cap(ray, t, s->maximum) : or_check_cap(ray, t, 1.0)) t_out[n++] = t;
  return n;
}

/* sphere.rs:47-62 / plane.rs:53-60 / cube.rs:71-93 / cylinder.rs:92-120 /
 * cone.rs:92-133. Returns the number of roots, in the reference's push order. */
int or_local_intersect(const oshape* s, const oray* ray, double t_out[OR_MAX_LOCAL_XS]) {
  const ot3 o = ray->origin, d = ray->direction;
  if (s->kind == RT_SHAPE_CUBE) {
    double xtmin, xtmax, ytmin, ytmax, ztmin, ztmax;
    or_cube_check_axis(o.x, d.x, &xtmin, &xtmax);
    or_cube_check_axis(o.y, d.y, &ytmin, &ytmax);
    or_cube_check_axis(o.z, d.z, &ztmin, &ztmax);
    double tmin = fmax(fmax(xtmin, ytmin), ztmin); /* f64::max ignores NaN like fmax */
    double tmax = fmin(fmin(xtmax, ytmax), ztmax);
    if (tmin > tmax) return 0;
    t_out[0] = tmin; t_out[1] = tmax;
    return 2;
  }
  if (s->kind == RT_SHAPE_CYLINDER) {
    double a = d.x * d.x + d.z * d.z; /* powi(2) = x*x */
    if (fabs(a) < OR_EPSILON) return or_intersect_caps(s, ray, t_out, 0);
    double b = 2.0 * o.x * d.x + 2.0 * o.z * d.z;
    double c = o.x * o.x + o.z * o.z - 1.0;
    double disc = b * b - 4.0 * a * c;
    if (disc < 0.0) return 0; /* no caps either (cylinder.rs:103-105) */
    double t0 = (-b - sqrt(disc)) / (2.0 * a);
    double t1 = (-b + sqrt(disc)) / (2.0 * a);
    int n = 0;
    double y0 = o.y + t0 * d.y;
    if (s->minimum < y0 && y0 < s->maximum) t_out[n++] = t0;
    double y1 = o.y + t1 * d.y;
    if (s->minimum < y1 && y1 < s->maximum) t_out[n++] = t1;
    return or_intersect_caps(s, ray, t_out, n);
  }
  if (s->kind == RT_SHAPE_CONE) {
    double a = d.x * d.x - d.y * d.y + d.z * d.z;
    double b = 2.0 * o.x * d.x - 2.0 * o.y * d.y + 2.0 * o.z * d.z;
    double c = o.x * o.x - o.y * o.y + o.z * o.z;
    if (fabs(a) < OR_EPSILON) {
      if (fabs(b) < OR_EPSILON) return or_intersect_caps(s, ray, t_out, 0);
      t_out[0] = -c / 2.0 * b; /* sic: (-c / 2) * b (cone.rs:104) */
      return or_intersect_caps(s, ray, t_out, 1);
    }
    double disc = b * b - 4.0 * a * c;
    if (disc < 0.0) return 0;
    double t0 = (-b - sqrt(disc)) / (2.0 * a);
    double t1 = (-b + sqrt(disc)) / (2.0 * a);
    int n = 0;
    double y0 = o.y + t0 * d.y;
    if (s->minimum < y0 && y0 < s->maximum) t_out[n++] = t0;
    double y1 = o.y + t1 * d.y;
    if (s->minimum < y1 && y1 < s->maximum) t_out[n++] = t1;
    return or_intersect_caps(s, ray, t_out, n);
  }
  if (s->kind == RT_SHAPE_SPHERE) {
    ot3 sphere_to_ray = or_sub(ray->origin, or_t3(0, 0, 0));
    double a = or_dot(ray->direction, ray->direction);
    double b = 2.0 * or_dot(ray->direction, sphere_to_ray);
    double c = or_dot(sphere_to_ray, sphere_to_ray) - 1.0;
    double discriminant = b * b - 4.0 * a * c;
    if (discriminant < 0.0) return 0;
    t_out[0] = (-b - sqrt(discriminant)) / (2.0 * a);
    t_out[1] = (-b + sqrt(discriminant)) / (2.0 * a);
    return 2;
  } else {
    if (fabs(ray->direction.y) < OR_EPSILON) return 0;
    t_out[0] = -ray->origin.y / ray->direction.y;
    return 1;
  }
}
/* geometry/mod.rs:46-49 + ray.rs:26-28 */
int or_shape_intersect(const oshape* s, const oray* r, double t_out[OR_MAX_LOCAL_XS], rt_stats* st) {
  oray local;
  local.origin = om_mul_point(&s->inverse, r->origin);
  local.direction = om_mul_vector(&s->inverse, r->direction);
  int n = or_local_intersect(s, &local, t_out);
  if (st) {
    if (s->kind == RT_SHAPE_SPHERE) { st->sphere_tests++; if (n) st->sphere_disc_ge0++; }
    else if (s->kind == RT_SHAPE_PLANE) st->plane_tests++;
    else st->other_tests++;
  }
  return n;
}
/* geometry/mod.rs:51-56 */
ot3 or_local_normal_at(const oshape* s, ot3 p) {
  switch (s->kind) {
    case RT_SHAPE_SPHERE: return or_sub(p, or_t3(0, 0, 0)); /* sphere.rs:64-67 */
    case RT_SHAPE_PLANE: return or_t3(0, 1, 0);              /* plane.rs:62-64 */
    case RT_SHAPE_CUBE: {                                     /* cube.rs:95-106 */
      double maxc = fmax(fmax(fabs(p.x), fabs(p.y)), fabs(p.z));
      if (or_equal(maxc, fabs(p.x))) return or_t3(p.x, 0.0, 0.0);
      if (or_equal(maxc, fabs(p.y))) return or_t3(0.0, p.y, 0.0);
      return or_t3(0.0, 0.0, p.z);
    }
    default: { /* cylinder.rs:122-130 / cone.rs:135-149 */
      double dist = p.x * p.x + p.z * p.z;
      if (dist < 1.0 && p.y >= s->maximum - OR_EPSILON) return or_t3(0, 1, 0);
      if (dist < 1.0 && p.y <= s->minimum + OR_EPSILON) return or_t3(0, -1, 0);
      if (s->kind == RT_SHAPE_CYLINDER) return or_t3(p.x, 0.0, p.z);
      double y = sqrt(p.x * p.x + p.z * p.z);
      if (p.y > 0.0) y = -y;
      return or_t3(p.x, y, p.z);
    }
  }
}
ot3 or_normal_at(const oshape* s, ot3 point) {
  ot3 local_point = om_mul_point(&s->inverse, point);
  ot3 local_normal = or_local_normal_at(s, local_point);
  ot3 world_normal = om_mul_vector(&s->inverse_t, local_normal);
  return or_normalize(world_normal);
}

/* ------------------------------------------------- geometry/intersection.rs */
/* :108-116 — stable merge sort by t (partial_cmp; NaN flagged, reference panics) */
static void or_merge(oxs* a, oxs* tmp, int lo, int mid, int hi) {
  int i = lo, j = mid, k = lo;
  while (i < mid && j < hi) {
    if (a[j].t < a[i].t) tmp[k++] = a[j++];
    else tmp[k++] = a[i++];
  }
  while (i < mid) tmp[k++] = a[i++];
  while (j < hi) tmp[k++] = a[j++];
  for (k = lo; k < hi; ++k) a[k] = tmp[k];
}
void or_sort_intersections(oxs* xs, int n) {
  for (int i = 0; i < n; ++i) if (isnan(xs[i].t)) g_nan_seen = 1;
  if (n < 2) return;
  oxs* tmp = (oxs*)malloc(sizeof(oxs) * n);
  for (int w = 1; w < n; w *= 2)
    for (int lo = 0; lo < n - w; lo += 2 * w) {
      int mid = lo + w, hi = lo + 2 * w < n ? lo + 2 * w : n;
      or_merge(xs, tmp, lo, mid, hi);
    }
  free(tmp);
}
/* world.rs:31-38: flat_map over objects, collect, intersections() (copy + sort) */
/* group.rs:49-58: Group::intersect returns nothing when the ray misses the
 * group's box, so none of its children (nested groups included) is
 * intersected; a flattened primitive is intersected iff the ray meets the box
 * of every group around it. */
static int or_group_gate(const oworld* w, int gate, const oray* r) {
  for (int g = gate - 1; g >= 0; g = w->groups[g].parent)
    if (!or_bbox_intersects(&w->groups[g].box, r)) return 0;
  return 1;
}
oxs* or_world_intersect(const oworld* w, const oray* r, int* n_out, rt_stats* st) {
  int cap = 8, n = 0;
  oxs* xs = (oxs*)malloc(sizeof(oxs) * cap);
  for (int i = 0; i < w->n; ++i) {
    if (w->objects[i].gate && !or_group_gate(w, w->objects[i].gate, r)) continue;
    double t[OR_MAX_LOCAL_XS];
    int k = or_shape_intersect(&w->objects[i], r, t, st);
    for (int j = 0; j < k; ++j) {
      if (n == cap) { cap *= 2; xs = (oxs*)realloc(xs, sizeof(oxs) * cap); }
      xs[n].t = t[j]; xs[n].obj = i; ++n;
    }
  }
  /* intersections(&xs): copy then sort (intersection.rs:108-116) */
  oxs* v = (oxs*)malloc(sizeof(oxs) * (n ? n : 1));
  if (n) memcpy(v, xs, sizeof(oxs) * n);
  free(xs);
  or_sort_intersections(v, n);
  *n_out = n;
  return v;
}
/* :118-120 */
int or_hit(const oxs* xs, int n) {
  for (int i = 0; i < n; ++i) if (xs[i].t >= 0.0) return i;
  return -1;
}
/* :122-125 */
static int or_shadow_hit(const oworld* w, const oxs* xs, int n) {
  for (int i = 0; i < n; ++i)
    if (xs[i].t >= 0.0 && w->objects[xs[i].obj].shadow) return i;
  return -1;
}
/* Intersection derived PartialEq (:10): t exact, object structural, u/v None */
static int or_xs_eq(const oworld* w, const oxs* a, const oxs* b) {
  return a->t == b->t && or_shape_equals(&w->objects[a->obj], &w->objects[b->obj]);
}
/* :53-105 */
ocomps or_prepare_computations(const oworld* w, const oxs* self, const oray* ray,
                               const oxs* xs, int n) {
  ocomps c;
  const oshape* obj = &w->objects[self->obj];
  ot3 point = or_add(ray->origin, or_scale(ray->direction, self->t)); /* ray.rs:22-24 */
  ot3 eyev = or_neg(ray->direction);
  ot3 normalv = or_normal_at(obj, point);
  int inside = 0;
  if (or_dot(normalv, eyev) < 0.0) { inside = 1; normalv = or_neg(normalv); }

  /* containers walk :63-90 */
  int* containers = (int*)malloc(sizeof(int) * (n + 1));
  int nc = 0;
  double n1 = -1.0, n2 = -1.0;
  for (int k = 0; k < n; ++k) {
    const oxs* i = &xs[k];
    int is_self = or_xs_eq(w, i, self);
    if (is_self) n1 = nc == 0 ? 1.0 : w->objects[containers[nc - 1]].material.refractive_index;
    int pos = -1;
    for (int q = 0; q < nc; ++q)
      if (or_shape_equals(&w->objects[containers[q]], &w->objects[i->obj])) { pos = q; break; }
    if (pos >= 0) {
      for (int q = pos; q < nc - 1; ++q) containers[q] = containers[q + 1];
      --nc;
    } else {
      containers[nc++] = i->obj;
    }
    if (is_self) {
      n2 = nc == 0 ? 1.0 : w->objects[containers[nc - 1]].material.refractive_index;
      break;
    }
  }
  free(containers);

  c.obj = self->obj;
  c.t = self->t;
  c.point = point;
  c.over_point = or_add(point, or_scale(normalv, OR_EPSILON));
  c.under_point = or_sub(point, or_scale(normalv, OR_EPSILON));
  c.eyev = eyev;
  c.normalv = normalv;
  c.inside = inside;
  c.reflectv = or_reflect(ray->direction, normalv);
  c.n1 = n1;
  c.n2 = n2;
  return c;
}
/* :147-162; powi(2) = q*q, powi(5) = x*((x*x)*(x*x)) (LLVM powi expansion /
 * compiler-rt __powidf2 give the same product sequence) */
double or_schlick(const ocomps* c) {
  double cosv = or_dot(c->eyev, c->normalv);
  if (c->n1 > c->n2) {
    double nn = c->n1 / c->n2;
    double sin2_t = nn * nn * (1.0 - cosv * cosv);
    if (sin2_t > 1.0) return 1.0;
    double cos_t = sqrt(1.0 - sin2_t);
    cosv = cos_t;
  }
  double q = (c->n1 - c->n2) / (c->n1 + c->n2);
  double r0 = q * q;
  double x = 1.0 - cosv;
  double x5 = x * ((x * x) * (x * x));
  return r0 + (1.0 - r0) * x5;
}

/* --------------------------------------------------------------- world.rs */
void or_world_init(oworld* w) { memset(w, 0, sizeof *w); }
void or_world_free(oworld* w) { free(w->objects); free(w->lights); free(w->groups); memset(w, 0, sizeof *w); }
int or_world_add_group(oworld* w, obbox box, int parent) {
  if (w->ng == w->capg) {
    w->capg = w->capg ? 2 * w->capg : 8;
    w->groups = (ogroup*)realloc(w->groups, sizeof(ogroup) * w->capg);
  }
  w->groups[w->ng].box = box;
  w->groups[w->ng].parent = parent;
  return w->ng++;
}
int or_world_add_object(oworld* w, const oshape* s) { /* :87-89 */
  if (w->n == w->cap) {
    w->cap = w->cap ? 2 * w->cap : 8;
    w->objects = (oshape*)realloc(w->objects, sizeof(oshape) * w->cap);
  }
  w->objects[w->n++] = *s;
  return w->n - 1;
}
int or_world_add_light(oworld* w, ot3 pos, ot3 intensity) { /* :83-85 */
  if (w->nl == w->capl) {
    w->capl = w->capl ? 2 * w->capl : 4;
    w->lights = (olight*)realloc(w->lights, sizeof(olight) * w->capl);
  }
  w->lights[w->nl].position = pos;
  w->lights[w->nl].intensity = intensity;
  return w->nl++;
}
/* :137-151 */
void or_world_default(oworld* w) {
  or_world_init(w);
  or_world_add_light(w, or_t3(-10, 10, -10), or_t3(1.0, 1.0, 1.0));
  oshape s1 = or_sphere_default();
  s1.material.color = or_t3(0.8, 1.0, 0.6);
  s1.material.diffuse = 0.7;
  s1.material.specular = 0.2;
  oshape s2 = or_sphere_default();
  omat sc = or_scaling(0.5, 0.5, 0.5);
  or_shape_set_transform(&s2, &sc);
  or_world_add_object(w, &s1);
  or_world_add_object(w, &s2);
}

enum { OR_RAY_PRIMARY = 0, OR_RAY_REFLECT = 1, OR_RAY_REFRACT = 2 };
static ot3 or_color_at_kind(const oworld* w, const oray* r, unsigned remaining, int kind, rt_stats* st);

/* :95-105 */
int or_is_shadowed(const oworld* w, ot3 point, const olight* light, rt_stats* st) {
  ot3 v = or_sub(light->position, point);
  double distance = or_magnitude(v);
  ot3 direction = or_normalize(v);
  oray r = {point, direction};
  int n;
  if (st) st->rays_shadow++;
  oxs* xs = or_world_intersect(w, &r, &n, st);
  int h = or_shadow_hit(w, xs, n);
  int res = h >= 0 && xs[h].t < distance;
  free(xs);
  return res;
}
/* :107-114 */
ot3 or_reflected_color(const oworld* w, const ocomps* c, unsigned remaining, rt_stats* st) {
  const omaterial* m = &w->objects[c->obj].material;
  if (or_equal(m->reflective, 0.0) || remaining == 0) return or_t3(0, 0, 0);
  oray rr = {c->over_point, c->reflectv};
  ot3 color = or_color_at_kind(w, &rr, remaining - 1, OR_RAY_REFLECT, st);
  return or_scale(color, m->reflective);
}
/* :116-134 */
ot3 or_refracted_color(const oworld* w, const ocomps* c, unsigned remaining, rt_stats* st) {
  const omaterial* m = &w->objects[c->obj].material;
  if (or_equal(m->transparency, 0.0) || remaining == 0) return or_t3(0, 0, 0);
  double n_ratio = c->n1 / c->n2;
  double cos_i = or_dot(c->eyev, c->normalv);
  double sin2_t = n_ratio * n_ratio * (1.0 - cos_i * cos_i);
  if (sin2_t > 1.0) return or_t3(0, 0, 0);
  double cos_t = sqrt(1.0 - sin2_t);
  ot3 direction = or_sub(or_scale(c->normalv, n_ratio * cos_i - cos_t), or_scale(c->eyev, n_ratio));
  oray rr = {c->under_point, direction};
  return or_scale(or_color_at_kind(w, &rr, remaining - 1, OR_RAY_REFRACT, st), m->transparency);
}
/* :40-68 */
ot3 or_shade_hit(const oworld* w, const ocomps* c, unsigned remaining, rt_stats* st) {
  const oshape* obj = &w->objects[c->obj];
  ot3 surface = or_t3(0.0, 0.0, 0.0); /* Sum = fold from (0,0,0), color.rs:96-103 */
  for (int l = 0; l < w->nl; ++l) {
    int shadowed = or_is_shadowed(w, c->over_point, &w->lights[l], st);
    ot3 lc = or_lighting(&obj->material, obj, &w->lights[l], c->over_point, c->eyev, c->normalv, shadowed);
    surface = or_add(surface, lc);
  }
  ot3 reflected = or_reflected_color(w, c, remaining, st);
  ot3 refracted = or_refracted_color(w, c, remaining, st);
  const omaterial* m = &obj->material;
  if (m->reflective > 0.0 && m->transparency > 0.0) {
    double reflectance = or_schlick(c);
    return or_add(or_add(surface, or_scale(reflected, reflectance)), or_scale(refracted, 1.0 - reflectance));
  }
  return or_add(or_add(surface, reflected), refracted);
}
/* :70-81 */
static ot3 or_color_at_kind(const oworld* w, const oray* r, unsigned remaining, int kind, rt_stats* st) {
  if (st) {
    if (kind == OR_RAY_PRIMARY) st->rays_primary++;
    else if (kind == OR_RAY_REFLECT) st->rays_reflect++;
    else st->rays_refract++;
  }
  int n;
  oxs* xs = or_world_intersect(w, r, &n, st);
  int h = or_hit(xs, n);
  ot3 res = or_t3(0.0, 0.0, 0.0);
  if (h >= 0) {
    ocomps c = or_prepare_computations(w, &xs[h], r, xs, n);
    res = or_shade_hit(w, &c, remaining, st);
  }
  free(xs);
  return res;
}
ot3 or_color_at(const oworld* w, const oray* r, unsigned remaining, rt_stats* st) {
  return or_color_at_kind(w, r, remaining, OR_RAY_PRIMARY, st);
}

/* -------------------------------------------------------------- camera.rs */
/* :33-55 */
void or_camera_new(ocamera* c, uint32_t hsize, uint32_t vsize, double fov) {
  double half_view = tan(fov / 2.0);
  double aspect = (double)hsize / (double)vsize;
  if (aspect >= 1.0) { c->half_width = half_view; c->half_height = half_view / aspect; }
  else { c->half_width = half_view * aspect; c->half_height = half_view; }
  c->pixel_size = c->half_width * 2.0 / (double)hsize;
  c->hsize = hsize; c->vsize = vsize; c->fov = fov;
  c->transform = om_identity(4);
  c->inverse = om_identity(4);
}
/* :128-131 */
int or_camera_set_transform(ocamera* c, const omat* t) {
  omat inv;
  int rc = om_inverse(t, &inv);
  if (rc != RT_OK) return rc;
  c->transform = *t;
  c->inverse = inv;
  return RT_OK;
}
/* :57-69 */
oray or_ray_for_pixel(const ocamera* c, uint32_t px, uint32_t py) {
  double xoffset = ((double)px + 0.5) * c->pixel_size;
  double yoffset = ((double)py + 0.5) * c->pixel_size;
  double world_x = c->half_width - xoffset;
  double world_y = c->half_height - yoffset;
  ot3 pixel = om_mul_point(&c->inverse, or_t3(world_x, world_y, -1.0));
  ot3 origin = om_mul_point(&c->inverse, or_t3(0, 0, 0));
  oray r;
  r.origin = origin;
  r.direction = or_normalize(or_sub(pixel, origin));
  return r;
}
/* :92-126 get_offsets */
static const double OR_AA_X1[] = {0.5, 0.5};
static const double OR_AA_X2[] = {0.25, 0.5, 0.75, 0.5};
static const double OR_AA_X4[] = {0.25, 0.25, 0.75, 0.25, 0.25, 0.75, 0.75, 0.75};
static const double OR_AA_X8[] = {0.25, 0.25, 0.5, 0.25, 0.75, 0.25, 0.25, 0.5,
                                  0.75, 0.5,  0.25, 0.75, 0.5, 0.75, 0.75, 0.75};
static const double OR_AA_X16[] = {0.125, 0.125, 0.375, 0.125, 0.625, 0.125, 0.875, 0.125,
                                   0.125, 0.375, 0.375, 0.375, 0.625, 0.375, 0.875, 0.375,
                                   0.125, 0.625, 0.375, 0.625, 0.625, 0.625, 0.875, 0.625,
                                   0.125, 0.875, 0.375, 0.875, 0.625, 0.875, 0.875, 0.875};
/* :71-90. Returns the number of rays (0 for an unsupported sample count). */
int or_rays_for_pixel(const ocamera* c, uint32_t px, uint32_t py, uint32_t aa_samples, oray* out) {
  const double* off;
  switch (aa_samples) {
    case 1: off = OR_AA_X1; break;
    case 2: off = OR_AA_X2; break;
    case 4: off = OR_AA_X4; break;
    case 8: off = OR_AA_X8; break;
    case 16: off = OR_AA_X16; break;
    default: return 0;
  }
  for (uint32_t i = 0; i < aa_samples; ++i) {
    double xoffset = ((double)px + off[2 * i]) * c->pixel_size;
    double yoffset = ((double)py + off[2 * i + 1]) * c->pixel_size;
    double world_x = c->half_width - xoffset;
    double world_y = c->half_height - yoffset;
    ot3 pixel = om_mul_point(&c->inverse, or_t3(world_x, world_y, -1.0));
    ot3 origin = om_mul_point(&c->inverse, or_t3(0, 0, 0));
    out[i].origin = origin;
    out[i].direction = or_normalize(or_sub(pixel, origin));
  }
  return (int)aa_samples;
}

/* ---------------------------------------------------------- image/ppm.rs */
/* :73-75: (v*255.0).round() as u8 — round half away from zero, saturating */
uint8_t or_scale_color_component(double v) {
  double s = round(v * 255.0);
  if (!(s > 0.0)) return 0; /* NaN and <= 0 */
  if (s >= 255.0) return 255;
  return (uint8_t)s;
}
/* :24-63 */
size_t or_canvas_to_ppm(const double* rgb, uint32_t w, uint32_t h, char* out, size_t cap) {
  size_t len = 0;
#define OR_EMIT(s, n)                              \
  do {                                             \
    if (out && len + (n) <= cap) memcpy(out + len, (s), (n)); \
    len += (n);                                    \
  } while (0)
  char hdr[64];
  int hn = snprintf(hdr, sizeof hdr, "P3\n%u %u\n255\n", w, h);
  OR_EMIT(hdr, (size_t)hn);
  char line[128];
  for (uint32_t j = 0; j < h; ++j) {
    size_t ll = 0;
    for (uint32_t i = 0; i < w; ++i) {
      const double* px = rgb + ((size_t)j * w + i) * 3;
      for (int idx = 0; idx < 3; ++idx) {
        char val[8];
        int vn = snprintf(val, sizeof val, "%u", (unsigned)or_scale_color_component(px[idx]));
        if (ll + (size_t)vn > 70) {
          size_t tl = ll;
          while (tl > 0 && line[tl - 1] == ' ') --tl; /* trim_end */
          OR_EMIT(line, tl);
          OR_EMIT("\n", 1);
          ll = 0;
        }
        memcpy(line + ll, val, vn); ll += vn;
        if (idx < 2) line[ll++] = ' ';
      }
      if (i < w - 1) line[ll++] = ' ';
    }
    OR_EMIT(line, ll);
    OR_EMIT("\n", 1);
  }
#undef OR_EMIT
  return len;
}

/* ------------------------------------------------------------ flat C API */
oworld* oracle_world_new(void) { oworld* w = (oworld*)malloc(sizeof(oworld)); or_world_init(w); return w; }
void oracle_world_free(oworld* w) { if (w) { or_world_free(w); free(w); } }
void oracle_world_set_default(oworld* w) { or_world_free(w); or_world_default(w); }

static ot3 or_v3(const double* v) { return or_t3(v[0], v[1], v[2]); }

/* Build a shape as the reference API would: Default, material fields, pattern
 * with set_transform, shape set_transform (once, from identity). The desc's
 * `inverse` is ignored: the oracle recomputes it with its own restatement. */
int oracle_world_add_desc(oworld* w, const rt_shape_desc* d) {
  oshape s;
  if (d->kind == RT_SHAPE_SPHERE) s = or_sphere_default();
  else if (d->kind == RT_SHAPE_PLANE) s = or_plane_default();
  else if (d->kind == RT_SHAPE_CUBE) s = or_cube_default();
  else if (d->kind == RT_SHAPE_CYLINDER) s = or_cylinder_new(d->minimum, d->maximum, d->closed);
  else if (d->kind == RT_SHAPE_CONE) s = or_cone_new(d->minimum, d->maximum, d->closed);
  else return RT_ERR_UNSUPPORTED_SHAPE;
  omaterial* m = &s.material;
  m->color = or_v3(d->color);
  m->ambient = d->ambient; m->diffuse = d->diffuse; m->specular = d->specular;
  m->shininess = d->shininess; m->reflective = d->reflective;
  m->transparency = d->transparency; m->refractive_index = d->refractive_index;
  if (d->pattern_kind != RT_PATTERN_NONE) {
    m->has_pattern = 1;
    m->pattern = or_pattern(d->pattern_kind, or_v3(d->pattern_a), or_v3(d->pattern_b));
    /* a bitwise-identity transform stands for "set_transform never called" */
    omat pt = om_from(4, 4, d->pattern_transform);
    omat id = om_identity(4);
    if (memcmp(d->pattern_transform, id.e, sizeof id.e) != 0) or_pattern_set_transform(&m->pattern, &pt);
  }
  omat t = om_from(4, 4, d->transform);
  omat id = om_identity(4);
  if (memcmp(d->transform, id.e, sizeof id.e) != 0) {
    int rc = or_shape_set_transform(&s, &t);
    if (rc != RT_OK) return rc;
  }
  s.shadow = d->casts_shadow ? 1 : 0;
  or_world_add_object(w, &s);
  return RT_OK;
}
/* A Group (rt_group_desc: its box, the enclosing group) and the innermost
 * group of the shape added last (the flattened World, group.rs). */
int oracle_world_add_group(oworld* w, const rt_group_desc* g) {
  if (g->parent < -1 || g->parent >= w->ng) return RT_ERR_INVALID_ARGUMENT;
  obbox b = {or_v3(g->min), or_v3(g->max)};
  return or_world_add_group(w, b, g->parent);
}
int oracle_world_set_last_group(oworld* w, int group) {
  if (w->n == 0 || group < -1 || group >= w->ng) return RT_ERR_INVALID_ARGUMENT;
  w->objects[w->n - 1].gate = group + 1;
  return RT_OK;
}
int oracle_world_export_desc(const oworld* w, rt_shape_desc* out, size_t cap) {
  for (int i = 0; i < w->n && (size_t)i < cap; ++i) {
    const oshape* s = &w->objects[i];
    rt_shape_desc* d = &out[i];
    memset(d, 0, sizeof *d);
    d->kind = s->kind; d->casts_shadow = s->shadow;
    d->minimum = s->minimum; d->maximum = s->maximum; d->closed = s->closed;
    memcpy(d->transform, s->transform.e, sizeof d->transform);
    memcpy(d->inverse, s->inverse.e, sizeof d->inverse);
    const omaterial* m = &s->material;
    d->color[0] = m->color.x; d->color[1] = m->color.y; d->color[2] = m->color.z;
    d->ambient = m->ambient; d->diffuse = m->diffuse; d->specular = m->specular;
    d->shininess = m->shininess; d->reflective = m->reflective;
    d->transparency = m->transparency; d->refractive_index = m->refractive_index;
    d->pattern_kind = m->has_pattern ? m->pattern.kind : RT_PATTERN_NONE;
    if (m->has_pattern) {
      d->pattern_a[0] = m->pattern.a.x; d->pattern_a[1] = m->pattern.a.y; d->pattern_a[2] = m->pattern.a.z;
      d->pattern_b[0] = m->pattern.b.x; d->pattern_b[1] = m->pattern.b.y; d->pattern_b[2] = m->pattern.b.z;
      memcpy(d->pattern_transform, m->pattern.transform.e, sizeof d->pattern_transform);
      memcpy(d->pattern_inverse, m->pattern.inverse.e, sizeof d->pattern_inverse);
    } else {
      omat id = om_identity(4);
      memcpy(d->pattern_transform, id.e, sizeof id.e);
      memcpy(d->pattern_inverse, id.e, sizeof id.e);
    }
  }
  return w->n;
}
int oracle_world_add_light(oworld* w, const double pos[3], const double intensity[3]) {
  return or_world_add_light(w, or_v3(pos), or_v3(intensity));
}
int oracle_matrix_inverse(const double m[16], double out[16]) {
  omat a = om_from(4, 4, m), inv;
  int rc = om_inverse(&a, &inv);
  if (rc == RT_OK) memcpy(out, inv.e, sizeof(double) * 16);
  return rc;
}
int oracle_camera_init(uint32_t hsize, uint32_t vsize, double fov, const double transform[16],
                       rt_camera_desc* out) {
  ocamera c;
  or_camera_new(&c, hsize, vsize, fov);
  if (transform) {
    omat t = om_from(4, 4, transform);
    int rc = or_camera_set_transform(&c, &t);
    if (rc != RT_OK) return rc;
  }
  out->hsize = hsize; out->vsize = vsize;
  out->pixel_size = c.pixel_size; out->half_width = c.half_width; out->half_height = c.half_height;
  memcpy(out->inverse, c.inverse.e, sizeof out->inverse);
  return RT_OK;
}
void oracle_color_at(const oworld* w, const double ray[6], uint32_t remaining, double out[3],
                     rt_stats* st) {
  oray r = {or_v3(ray), or_v3(ray + 3)};
  ot3 c = or_color_at(w, &r, remaining, st);
  out[0] = c.x; out[1] = c.y; out[2] = c.z;
}
int oracle_is_shadowed(const oworld* w, const double p[3], uint32_t light) {
  if ((int)light >= w->nl) return -1;
  return or_is_shadowed(w, or_v3(p), &w->lights[light], NULL);
}
void oracle_hit(const oworld* w, const double ray[6], double o[24]) {
  oray r = {or_v3(ray), or_v3(ray + 3)};
  int n;
  oxs* xs = or_world_intersect(w, &r, &n, NULL);
  int h = or_hit(xs, n);
  memset(o, 0, sizeof(double) * 24);
  o[0] = -1.0;
  if (h >= 0) {
    ocomps c = or_prepare_computations(w, &xs[h], &r, xs, n);
    o[0] = c.obj; o[1] = c.t;
    o[2] = c.point.x; o[3] = c.point.y; o[4] = c.point.z;
    o[5] = c.over_point.x; o[6] = c.over_point.y; o[7] = c.over_point.z;
    o[8] = c.under_point.x; o[9] = c.under_point.y; o[10] = c.under_point.z;
    o[11] = c.eyev.x; o[12] = c.eyev.y; o[13] = c.eyev.z;
    o[14] = c.normalv.x; o[15] = c.normalv.y; o[16] = c.normalv.z;
    o[17] = c.inside;
    o[18] = c.reflectv.x; o[19] = c.reflectv.y; o[20] = c.reflectv.z;
    o[21] = c.n1; o[22] = c.n2; o[23] = or_schlick(&c);
  }
  free(xs);
}

typedef struct {
  const oworld* w;
  ocamera cam;
  uint32_t max_depth, aa;
  const uint32_t* rows;
  const uint32_t* pix; /* oracle_render_pixels: (x, y) pairs instead of rows */
  uint32_t i0, i1; /* indices into the row (pixel) list */
  double* out;
  rt_stats st;
} or_job;

static ot3 or_pixel_color(or_job* j, uint32_t x, uint32_t y) {
  if (j->aa <= 1) { /* Camera::render (camera.rs:141-143) */
    oray r = or_ray_for_pixel(&j->cam, x, y);
    return or_color_at(j->w, &r, j->max_depth, &j->st);
  }
  /* render_multithreaded (camera.rs:176-185) + Color::average (color.rs:26-33) */
  oray rays[16];
  int n = or_rays_for_pixel(&j->cam, x, y, j->aa, rays);
  ot3 c = or_t3(0, 0, 0);
  for (int s = 0; s < n; ++s) c = or_add(c, or_color_at(j->w, &rays[s], j->max_depth, &j->st));
  return or_scale(c, 1.0 / (double)n);
}

static void* or_render_worker(void* arg) {
  or_job* j = (or_job*)arg;
  for (uint32_t i = j->i0; i < j->i1; ++i) {
    if (j->pix) {
      ot3 c = or_pixel_color(j, j->pix[2 * (size_t)i], j->pix[2 * (size_t)i + 1]);
      double* px = j->out + (size_t)i * 3;
      px[0] = c.x; px[1] = c.y; px[2] = c.z;
      continue;
    }
    uint32_t y = j->rows[i];
    for (uint32_t x = 0; x < j->cam.hsize; ++x) {
      ot3 c = or_pixel_color(j, x, y);
      double* px = j->out + ((size_t)i * j->cam.hsize + x) * 3;
      px[0] = c.x; px[1] = c.y; px[2] = c.z;
    }
  }
  return NULL;
}

static int or_render_list(const oworld* w, const rt_camera_desc* cam, uint32_t max_depth, uint32_t aa_samples,
                          const uint32_t* rows, const uint32_t* pix, uint32_t n_rows, uint32_t nthreads,
                          double* out_rgb, rt_stats* st);
int oracle_render_rows(const oworld* w, const rt_camera_desc* cam, uint32_t max_depth,
                       uint32_t aa_samples, const uint32_t* rows, uint32_t n_rows, uint32_t nthreads,
                       double* out_rgb, rt_stats* st) {
  return or_render_list(w, cam, max_depth, aa_samples, rows, NULL, n_rows, nthreads, out_rgb, st);
}
/* Pixels (x, y) = pix[2i], pix[2i + 1] of the frame, each as Camera::render
   (or render_multithreaded) computes it, into out_rgb[i]; the pixel list is
   split over the threads in contiguous blocks. Sampling a large frame (C5) at
   scattered pixels costs a fraction of whole rows. */
int oracle_render_pixels(const oworld* w, const rt_camera_desc* cam, uint32_t max_depth, uint32_t aa_samples,
                         const uint32_t* pix, uint32_t n_pix, uint32_t nthreads, double* out_rgb, rt_stats* st) {
  if (!pix && n_pix) return RT_ERR_INVALID_ARGUMENT;
  for (uint32_t i = 0; i < n_pix; ++i)
    if (pix[2 * (size_t)i] >= cam->hsize || pix[2 * (size_t)i + 1] >= cam->vsize) return RT_ERR_INVALID_ARGUMENT;
  return or_render_list(w, cam, max_depth, aa_samples, NULL, pix, n_pix, nthreads, out_rgb, st);
}
static int or_render_list(const oworld* w, const rt_camera_desc* cam, uint32_t max_depth, uint32_t aa_samples,
                          const uint32_t* rows, const uint32_t* pix, uint32_t n_rows, uint32_t nthreads,
                          double* out_rgb, rt_stats* st) {
  if (!(aa_samples == 1 || aa_samples == 2 || aa_samples == 4 || aa_samples == 8 || aa_samples == 16))
    return RT_ERR_INVALID_ARGUMENT;
  ocamera c;
  memset(&c, 0, sizeof c);
  c.hsize = cam->hsize; c.vsize = cam->vsize;
  c.pixel_size = cam->pixel_size; c.half_width = cam->half_width; c.half_height = cam->half_height;
  c.inverse = om_from(4, 4, cam->inverse);
  uint32_t* own = NULL;
  if (!rows && !pix) {
    own = (uint32_t*)malloc(sizeof(uint32_t) * (n_rows ? n_rows : 1));
    for (uint32_t i = 0; i < n_rows; ++i) own[i] = i;
    rows = own;
  }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > n_rows && n_rows > 0) nthreads = n_rows;
  or_job* jobs = (or_job*)calloc(nthreads, sizeof(or_job));
  pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
  uint32_t per = n_rows / nthreads; /* camera.rs:157, last block takes the rest :169-172 */
  for (uint32_t t = 0; t < nthreads; ++t) {
    jobs[t].w = w; jobs[t].cam = c; jobs[t].max_depth = max_depth; jobs[t].aa = aa_samples; jobs[t].rows = rows;
    jobs[t].pix = pix;
    jobs[t].i0 = t * per; jobs[t].i1 = (t == nthreads - 1) ? n_rows : (t + 1) * per;
    jobs[t].out = out_rgb;
    if (nthreads == 1) or_render_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, or_render_worker, &jobs[t]);
  }
  if (st) memset(st, 0, sizeof *st);
  for (uint32_t t = 0; t < nthreads; ++t) {
    if (nthreads > 1) pthread_join(th[t], NULL);
    if (st) {
      st->rays_primary += jobs[t].st.rays_primary; st->rays_reflect += jobs[t].st.rays_reflect;
      st->rays_refract += jobs[t].st.rays_refract; st->rays_shadow += jobs[t].st.rays_shadow;
      st->sphere_tests += jobs[t].st.sphere_tests; st->plane_tests += jobs[t].st.plane_tests;
      st->sphere_disc_ge0 += jobs[t].st.sphere_disc_ge0; st->other_tests += jobs[t].st.other_tests;
    }
  }
  free(jobs); free(th); free(own);
  return RT_OK;
}
size_t oracle_canvas_to_ppm(const double* rgb, uint32_t w, uint32_t h, char* out, size_t cap) {
  return or_canvas_to_ppm(rgb, w, h, out, cap);
}

/* ABI sizes for the ctypes wrapper (oracle/pyoracle.py) */
size_t oracle_sizeof_shape_desc(void) { return sizeof(rt_shape_desc); }
size_t oracle_sizeof_camera_desc(void) { return sizeof(rt_camera_desc); }
size_t oracle_sizeof_stats(void) { return sizeof(rt_stats); }
