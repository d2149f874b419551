/*
 * rt_oracle.h — CPU parity ORACLE for the render hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This is a plain-C restatement of the reference
 * Rust renderer tlinford/raytracer-challenge-rs (read as text, never copied),
 * following the reference's algorithm literally: every object is intersected,
 * the intersection list is collected and sorted, `hit` takes the first t >= 0,
 * `prepare_computations` walks the sorted list with the `containers` stack and
 * structural shape equality, and `color_at` recurses. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may link or call
 * it, and only as the checker / CPU baseline — never as the product path.
 *
 * Parity pin: the reference's own known-answer tests (oracle/kat.c transcribes
 * every one on this path; they pass at the reference's 1e-5 tolerance). The
 * reference cannot be built here (Rust toolchain absent), so no reference
 * binary output exists; see DESIGN.md "Oracle".
 *
 * Build: -O2 -ffp-contract=off, no -ffast-math (see oracle/Makefile).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/rt_render.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OR_EPSILON 0.00001 /* raytracer/src/lib.rs:18 */

typedef struct { double x, y, z; } ot3; /* Point / Vector / Color */

typedef struct { int rows, cols; double e[16]; } omat; /* Matrix (<= 4x4) */

typedef struct { ot3 origin, direction; } oray;

typedef struct { ot3 min, max; } obbox;

typedef struct {
  int kind; /* RT_PATTERN_* */
  ot3 a, b;
  omat transform, inverse;
} opattern;

typedef struct {
  ot3 color;
  double ambient, diffuse, specular, shininess;
  double reflective, transparency, refractive_index;
  int has_pattern;
  opattern pattern;
} omaterial;

typedef struct {
  int kind; /* RT_SHAPE_* */
  omat transform, inverse, inverse_t;
  omaterial material;
  obbox bbox;
  int shadow;
  double minimum, maximum; /* Cylinder / Cone (cylinder.rs:12-18, cone.rs:12-18) */
  int closed;
  int gate; /* 1 + the innermost Group around the shape (oworld.groups), 0: none */
} oshape;
typedef struct { obbox box; int parent; } ogroup; /* a Group's bounding box; parent: enclosing group, -1 none */

typedef struct { ot3 position, intensity; } olight;

typedef struct {
  oshape* objects; /* the primitives, Groups flattened (group.rs:49-58 visits children in order) */
  int n, cap;
  olight* lights;
  int nl, capl;
  ogroup* groups;
  int ng, capg;
} oworld;

typedef struct { double t; int obj; } oxs; /* Intersection (u, v are None) */

typedef struct {
  int obj;
  double t;
  ot3 point, over_point, under_point, eyev, normalv;
  int inside;
  ot3 reflectv;
  double n1, n2;
} ocomps;

typedef struct {
  uint32_t hsize, vsize;
  double fov;
  omat transform, inverse;
  double pixel_size, half_width, half_height;
} ocamera;

/* ---- math (matrix.rs, transform.rs, vector.rs, point.rs, color.rs) ---- */
int or_equal(double a, double b);
ot3 or_t3(double x, double y, double z);
ot3 or_add(ot3 a, ot3 b);
ot3 or_sub(ot3 a, ot3 b);
ot3 or_neg(ot3 a);
ot3 or_scale(ot3 a, double s);
ot3 or_hadamard(ot3 a, ot3 b);
double or_dot(ot3 a, ot3 b);
ot3 or_cross(ot3 a, ot3 b);
double or_magnitude(ot3 a);
ot3 or_normalize(ot3 a);
ot3 or_reflect(ot3 v, ot3 n);
int or_t3_eq(ot3 a, ot3 b);

omat om_zero(int r, int c);
omat om_identity(int n);
omat om_from(int r, int c, const double* e);
double om_at(const omat* m, int i, int j);
omat om_mul(const omat* a, const omat* b);
ot3 om_mul_point(const omat* m, ot3 p);
ot3 om_mul_vector(const omat* m, ot3 v);
omat om_transpose(const omat* m);
double om_determinant(const omat* m);
omat om_submatrix(const omat* m, int row, int col);
double om_minor(const omat* m, int row, int col);
double om_cofactor(const omat* m, int row, int col);
int om_is_invertible(const omat* m);
int om_inverse(const omat* m, omat* out);
int om_eq(const omat* a, const omat* b);

omat or_translation(double x, double y, double z);
omat or_scaling(double x, double y, double z);
omat or_rotation_x(double r);
omat or_rotation_y(double r);
omat or_rotation_z(double r);
omat or_shearing(double xy, double xz, double yx, double yz, double zx, double zy);
omat or_view_transform(ot3 from, ot3 to, ot3 up);

/* ---- scene ---- */
omaterial or_material_default(void);
opattern or_pattern(int kind, ot3 a, ot3 b);
void or_pattern_set_transform(opattern* p, const omat* t);
ot3 or_pattern_color_at(const opattern* p, ot3 pattern_point);
ot3 or_pattern_color_at_shape(const opattern* p, const oshape* s, ot3 world_point);
oshape or_sphere_default(void);
oshape or_sphere_glass(void);
oshape or_plane_default(void);
oshape or_cube_default(void);
oshape or_cylinder_new(double minimum, double maximum, int closed);
oshape or_cone_new(double minimum, double maximum, int closed);
int or_shape_set_transform(oshape* s, const omat* t);
int or_shape_equals(const oshape* a, const oshape* b);

void or_world_init(oworld* w);
void or_world_free(oworld* w);
int or_world_add_object(oworld* w, const oshape* s);
int or_world_add_light(oworld* w, ot3 pos, ot3 intensity);
void or_world_default(oworld* w);

/* ---- hot path (world.rs, geometry/{mod,intersection,shape}.rs, material.rs, camera.rs) ---- */
#define OR_MAX_LOCAL_XS 4 /* most intersections one local_intersect returns (cylinder/cone) */
int or_local_intersect(const oshape* s, const oray* local, double t_out[OR_MAX_LOCAL_XS]);
int or_shape_intersect(const oshape* s, const oray* r, double t_out[OR_MAX_LOCAL_XS], rt_stats* st);
oxs* or_world_intersect(const oworld* w, const oray* r, int* n_out, rt_stats* st);
int or_bbox_intersects(const obbox* b, const oray* r);
int or_world_add_group(oworld* w, obbox box, int parent);
void or_sort_intersections(oxs* xs, int n);
int or_hit(const oxs* xs, int n); /* index into xs or -1 */
ot3 or_local_normal_at(const oshape* s, ot3 local_point);
ot3 or_normal_at(const oshape* s, ot3 point);
ocomps or_prepare_computations(const oworld* w, const oxs* hit, const oray* r,
                               const oxs* xs, int n);
double or_schlick(const ocomps* c);
ot3 or_lighting(const omaterial* m, const oshape* obj, const olight* light,
                ot3 point, ot3 eyev, ot3 normalv, int in_shadow);
int or_is_shadowed(const oworld* w, ot3 point, const olight* light, rt_stats* st);
ot3 or_shade_hit(const oworld* w, const ocomps* c, unsigned remaining, rt_stats* st);
ot3 or_color_at(const oworld* w, const oray* r, unsigned remaining, rt_stats* st);
ot3 or_reflected_color(const oworld* w, const ocomps* c, unsigned remaining, rt_stats* st);
ot3 or_refracted_color(const oworld* w, const ocomps* c, unsigned remaining, rt_stats* st);

void or_camera_new(ocamera* c, uint32_t hsize, uint32_t vsize, double fov);
int or_camera_set_transform(ocamera* c, const omat* t);
oray or_ray_for_pixel(const ocamera* c, uint32_t px, uint32_t py);
int or_rays_for_pixel(const ocamera* c, uint32_t px, uint32_t py, uint32_t aa_samples, oray* out);

uint8_t or_scale_color_component(double v);
size_t or_canvas_to_ppm(const double* rgb, uint32_t w, uint32_t h, char* out, size_t cap);

/* ---- flat C API used by the Python tests / bench (ctypes) ---- */
oworld* oracle_world_new(void);
void oracle_world_free(oworld* w);
int oracle_world_add_desc(oworld* w, const rt_shape_desc* d);
int oracle_world_add_light(oworld* w, const double pos[3], const double intensity[3]);
void oracle_world_set_default(oworld* w);
int oracle_world_export_desc(const oworld* w, rt_shape_desc* out, size_t cap);
int oracle_matrix_inverse(const double m[16], double out[16]);
int oracle_camera_init(uint32_t hsize, uint32_t vsize, double fov,
                       const double transform[16], rt_camera_desc* out);
void oracle_color_at(const oworld* w, const double ray[6], uint32_t remaining,
                     double out[3], rt_stats* st);
int oracle_is_shadowed(const oworld* w, const double p[3], uint32_t light);
void oracle_hit(const oworld* w, const double ray[6], double out24[24]);
/* Render rows [0, n_rows) (or the explicit list `rows` of n_rows rows when
 * rows != NULL) into out_rgb (n_rows*hsize*3, rows in the given order) with
 * nthreads threads in contiguous row blocks (camera.rs:150-217).
 * aa_samples == 1: `Camera::render` (camera.rs:133-148, ray_for_pixel);
 * 2/4/8/16: `render_multithreaded` with `rays_for_pixel` + `Color::average`. */
int oracle_render_rows(const oworld* w, const rt_camera_desc* cam, uint32_t max_depth,
                       uint32_t aa_samples, const uint32_t* rows, uint32_t n_rows,
                       uint32_t nthreads, double* out_rgb, rt_stats* st);
/* The pixels (pix[2i], pix[2i+1]) = (x, y), each as oracle_render_rows
 * computes it, into out_rgb (n_pix*3); blocks of the list per thread. */
int oracle_render_pixels(const oworld* w, const rt_camera_desc* cam, uint32_t max_depth, uint32_t aa_samples,
                         const uint32_t* pix, uint32_t n_pix, uint32_t nthreads, double* out_rgb, rt_stats* st);
size_t oracle_canvas_to_ppm(const double* rgb, uint32_t w, uint32_t h, char* out, size_t cap);
int oracle_nan_seen(void);

#ifdef __cplusplus
}
#endif
#endif
