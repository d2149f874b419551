/*
 * kat.c — the reference's own known-answer tests for the render path,
 * transcribed against the C oracle (TEST INFRASTRUCTURE; see rt_oracle.h).
 *
 * Each case names the reference test (file:line of the #[test] fn). Values and
 * tolerance (1e-5, lib.rs:18-22) are the reference's. Output: one line per
 * case, "ok <name>" or "FAIL <name>: <detail>", then "KAT <passed>/<total>".
 * Exit status 0 iff every case passes. tests/test_oracle_kat.py drives it.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_oracle.h"

static int g_total = 0, g_failed = 0;
static const char* g_case = "";
static int g_case_failed = 0;

#define CASE(name) for (int _once = (begin_case(name), 1); _once; _once = 0, end_case())
static void begin_case(const char* n) { g_case = n; g_case_failed = 0; ++g_total; }
static void end_case(void) {
  if (g_case_failed) ++g_failed; else printf("ok %s\n", g_case);
}
static void fail(const char* what, int line) {
  if (!g_case_failed) printf("FAIL %s: %s (kat.c:%d)\n", g_case, what, line);
  g_case_failed = 1;
}
#define CHECK(c) do { if (!(c)) fail(#c, __LINE__); } while (0)
#define CHECK_EQ(a, b) CHECK(or_equal((a), (b)))
#define CHECK_T3(a, X, Y, Z) CHECK(or_t3_eq((a), or_t3((X), (Y), (Z))))

static omat M4(const double* e) { return om_from(4, 4, e); }
static oray R(double ox, double oy, double oz, double dx, double dy, double dz) {
  oray r = {or_t3(ox, oy, oz), or_t3(dx, dy, dz)};
  return r;
}
static void set_tf(oshape* s, omat t) { or_shape_set_transform(s, &t); }
/* local_intersect with a normalised direction (the shape tests normalise) */
static int local_xs(const oshape* s, ot3 o, ot3 d, int normalise, double t[OR_MAX_LOCAL_XS]) {
  oray r = {o, normalise ? or_normalize(d) : d};
  return or_local_intersect(s, &r, t);
}
static int count_intersect(const oshape* s, oray r, double t[OR_MAX_LOCAL_XS]) { return or_shape_intersect(s, &r, t, NULL); }

int main(void) {
  const double S2 = sqrt(2.0) / 2.0;
  const double S3 = sqrt(3.0) / 3.0;
  const double PI = 3.14159265358979323846;

  /* -------------------------------------------------------------- cube.rs */
  CASE("ray_intersects_cube") { /* cube.rs:114-148 */
    oshape c = or_cube_default();
    const double tc[7][8] = {{5, 0.5, 0, -1, 0, 0, 4, 6},  {-5, 0.5, 0, 1, 0, 0, 4, 6},
                             {0.5, 5, 0, 0, -1, 0, 4, 6},  {0.5, -5, 0, 0, 1, 0, 4, 6},
                             {0.5, 0, 5, 0, 0, -1, 4, 6},  {0.5, 0, -5, 0, 0, 1, 4, 6},
                             {0, 0.5, 0, 0, 0, 1, -1, 1}};
    for (int i = 0; i < 7; ++i) {
      double t[OR_MAX_LOCAL_XS];
      int n = local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 0, t);
      CHECK(n == 2); CHECK_EQ(t[0], tc[i][6]); CHECK_EQ(t[1], tc[i][7]);
    }
  }
  CASE("ray_misses_cube") { /* cube.rs:150-181 */
    oshape c = or_cube_default();
    const double tc[6][6] = {{-2, 0, 0, 0.2673, 0.5345, 0.8018}, {0, -2, 0, 0.8018, 0.2673, 0.5345},
                             {0, 0, -2, 0.5345, 0.8018, 0.2673}, {2, 0, 2, 0, 0, -1},
                             {0, 2, 2, 0, -1, 0},                {2, 2, 0, -1, 0, 0}};
    for (int i = 0; i < 6; ++i) {
      double t[OR_MAX_LOCAL_XS];
      CHECK(local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 0, t) == 0);
    }
  }
  CASE("normal_on_cube_surface") { /* cube.rs:183-214 */
    oshape c = or_cube_default();
    const double tc[8][6] = {{1, 0.5, -0.8, 1, 0, 0},   {-1, -0.2, -0.9, -1, 0, 0}, {-0.4, 1, -0.1, 0, 1, 0},
                             {0.3, -1, -0.7, 0, -1, 0}, {-0.6, 0.3, 1, 0, 0, 1},    {0.4, 0.4, -1, 0, 0, -1},
                             {1, 1, 1, 1, 0, 0},        {-1, -1, -1, -1, 0, 0}};
    for (int i = 0; i < 8; ++i)
      CHECK_T3(or_local_normal_at(&c, or_t3(tc[i][0], tc[i][1], tc[i][2])), tc[i][3], tc[i][4], tc[i][5]);
  }
  CASE("cube_bounding_box") { /* cube.rs:216-222 */
    oshape c = or_cube_default();
    CHECK_T3(c.bbox.min, -1, -1, -1); CHECK_T3(c.bbox.max, 1, 1, 1);
  }

  /* ---------------------------------------------------------- cylinder.rs */
  CASE("ray_misses_cylinder") { /* cylinder.rs:138-152 */
    oshape c = or_cylinder_new(-INFINITY, INFINITY, 0);
    const double tc[3][6] = {{1, 0, 0, 0, 1, 0}, {0, 0, 0, 0, 1, 0}, {0, 0, -5, 1, 1, 1}};
    for (int i = 0; i < 3; ++i) {
      double t[OR_MAX_LOCAL_XS];
      CHECK(local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 0, t) == 0);
    }
  }
  CASE("ray_strikes_cylinder") { /* cylinder.rs:154-196 */
    oshape c = or_cylinder_new(-INFINITY, INFINITY, 0);
    const double tc[3][8] = {{1, 0, -5, 0, 0, 1, 5, 5}, {0, 0, -5, 0, 0, 1, 4, 6},
                             {0.5, 0, -5, 0.1, 1, 1, 6.80798, 7.08872}};
    for (int i = 0; i < 3; ++i) {
      double t[OR_MAX_LOCAL_XS];
      int n = local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 1, t);
      CHECK(n == 2); CHECK_EQ(t[0], tc[i][6]); CHECK_EQ(t[1], tc[i][7]);
    }
  }
  CASE("normal_vector_on_cylinder") { /* cylinder.rs:198-212 */
    oshape c = or_cylinder_new(-INFINITY, INFINITY, 0);
    const double tc[4][6] = {{1, 0, 0, 1, 0, 0}, {0, 5, -1, 0, 0, -1}, {0, -2, 1, 0, 0, 1}, {-1, 1, 0, -1, 0, 0}};
    for (int i = 0; i < 4; ++i)
      CHECK_T3(or_local_normal_at(&c, or_t3(tc[i][0], tc[i][1], tc[i][2])), tc[i][3], tc[i][4], tc[i][5]);
  }
  CASE("default_cylinder_min_max_closed") { /* cylinder.rs:214-246 */
    oshape c = or_cylinder_new(-INFINITY, INFINITY, 0);
    CHECK(isinf(c.minimum) && c.minimum < 0); CHECK(isinf(c.maximum) && c.maximum > 0); CHECK(c.closed == 0);
  }
  CASE("intersect_constrained_cylinder") { /* cylinder.rs:220-240 */
    oshape c = or_cylinder_new(1.0, 2.0, 0);
    const double tc[6][7] = {{0, 1.5, 0, 0.1, 1, 0, 0}, {0, 3, -5, 0, 0, 1, 0}, {0, 0, -5, 0, 0, 1, 0},
                             {0, 2, -5, 0, 0, 1, 0},    {0, 1, -5, 0, 0, 1, 0}, {0, 1.5, -2, 0, 0, 1, 2}};
    for (int i = 0; i < 6; ++i) {
      double t[OR_MAX_LOCAL_XS];
      CHECK(local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 1, t) ==
            (int)tc[i][6]);
    }
  }
  CASE("intersect_caps_closed_cylinder") { /* cylinder.rs:248-264 */
    oshape c = or_cylinder_new(1.0, 2.0, 1);
    const double tc[5][6] = {{0, 3, 0, 0, -1, 0}, {0, 3, -2, 0, -1, 2}, {0, 4, -2, 0, -1, 1},
                             {0, 0, -2, 0, 1, 2}, {0, -1, -2, 0, 1, 1}};
    for (int i = 0; i < 5; ++i) {
      double t[OR_MAX_LOCAL_XS];
      CHECK(local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 1, t) == 2);
    }
  }
  CASE("normal_vector_on_cylinder_end_cap") { /* cylinder.rs:266-282 */
    oshape c = or_cylinder_new(1.0, 2.0, 1);
    const double tc[6][6] = {{0, 1, 0, 0, -1, 0},   {0.5, 1, 0, 0, -1, 0}, {0, 1, 0.5, 0, -1, 0},
                             {0, 2, 0, 0, 1, 0},    {0.5, 2, 0, 0, 1, 0},  {0, 2, 0.5, 0, 1, 0}};
    for (int i = 0; i < 6; ++i)
      CHECK_T3(or_local_normal_at(&c, or_t3(tc[i][0], tc[i][1], tc[i][2])), tc[i][3], tc[i][4], tc[i][5]);
  }
  CASE("bounded_cylinder_bounding_box") { /* cylinder.rs:296-302 */
    oshape c = or_cylinder_new(-5, 3, 0);
    CHECK_T3(c.bbox.min, -1, -5, -1); CHECK_T3(c.bbox.max, 1, 3, 1);
  }

  /* -------------------------------------------------------------- cone.rs */
  CASE("intersect_cone_with_ray") { /* cone.rs:155-192 */
    oshape c = or_cone_new(-INFINITY, INFINITY, 0);
    const double tc[3][8] = {{0, 0, -5, 0, 0, 1, 5, 5}, {0, 0, -5, 1, 1, 1, 8.66025, 8.66025},
                             {1, 1, -5, -0.5, -1, 1, 4.55006, 49.44994}};
    for (int i = 0; i < 3; ++i) {
      double t[OR_MAX_LOCAL_XS];
      int n = local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 1, t);
      CHECK(n == 2); CHECK_EQ(t[0], tc[i][6]); CHECK_EQ(t[1], tc[i][7]);
    }
  }
  CASE("intersect_cone_parallel_to_half") { /* book: ray parallel to one half, t = 0.35355 */
    /* The reference computes `-c / 2.0 * b` (cone.rs:104) and has no test for
     * this branch; the oracle keeps the reference's expression. */
    oshape c = or_cone_new(-INFINITY, INFINITY, 0);
    double t[OR_MAX_LOCAL_XS];
    int n = local_xs(&c, or_t3(0, 0, -1), or_t3(0, 1, 1), 1, t);
    CHECK(n == 1);
    oray r = {or_t3(0, 0, -1), or_normalize(or_t3(0, 1, 1))};
    double b = 2.0 * r.origin.x * r.direction.x - 2.0 * r.origin.y * r.direction.y + 2.0 * r.origin.z * r.direction.z;
    double cc = r.origin.x * r.origin.x - r.origin.y * r.origin.y + r.origin.z * r.origin.z;
    CHECK(t[0] == -cc / 2.0 * b);
  }
  CASE("intersect_cone_end_caps") { /* cone.rs:194-228 */
    oshape c = or_cone_new(-0.5, 0.5, 1);
    const double tc[3][7] = {{0, 0, -5, 0, 1, 0, 0}, {0, 0, -0.25, 0, 1, 1, 2}, {0, 0, -0.25, 0, 1, 0, 4}};
    for (int i = 0; i < 3; ++i) {
      double t[OR_MAX_LOCAL_XS];
      CHECK(local_xs(&c, or_t3(tc[i][0], tc[i][1], tc[i][2]), or_t3(tc[i][3], tc[i][4], tc[i][5]), 1, t) ==
            (int)tc[i][6]);
    }
  }
  CASE("computing_normal_vector_cone") { /* cone.rs:230-242 */
    oshape c = or_cone_new(-INFINITY, INFINITY, 0);
    CHECK_T3(or_local_normal_at(&c, or_t3(0, 0, 0)), 0, 0, 0);
    CHECK_T3(or_local_normal_at(&c, or_t3(1, 1, 1)), 1, -sqrt(2.0), 1);
    CHECK_T3(or_local_normal_at(&c, or_t3(-1, -1, 0)), -1, 1, 0);
  }
  CASE("bounded_cone_bounding_box") { /* cone.rs:256-262 */
    oshape c = or_cone_new(-5, 3, 0);
    CHECK_T3(c.bbox.min, -5, -5, -5); CHECK_T3(c.bbox.max, 5, 3, 5);
  }

  /* ------------------------------------------------- camera.rs (AA offsets) */
  CASE("rays_for_pixel_offsets") { /* camera.rs:71-126: X1 equals ray_for_pixel; Xn offsets */
    ocamera cam;
    or_camera_new(&cam, 201, 101, PI / 2.0);
    oray one = or_ray_for_pixel(&cam, 100, 50), rs[16];
    CHECK(or_rays_for_pixel(&cam, 100, 50, 1, rs) == 1);
    CHECK(memcmp(&one, &rs[0], sizeof one) == 0);
    CHECK(or_rays_for_pixel(&cam, 100, 50, 16, rs) == 16);
    CHECK(or_rays_for_pixel(&cam, 100, 50, 3, rs) == 0);
    CHECK(or_rays_for_pixel(&cam, 0, 0, 4, rs) == 4);
    /* sample (0.25, 0.25) of pixel (0,0): world (hw - 0.25*ps, hh - 0.25*ps, -1) */
    double wx = cam.half_width - 0.25 * cam.pixel_size, wy = cam.half_height - 0.25 * cam.pixel_size;
    CHECK_T3(rs[0].direction, or_normalize(or_t3(wx, wy, -1)).x, or_normalize(or_t3(wx, wy, -1)).y,
             or_normalize(or_t3(wx, wy, -1)).z);
  }

  /* ------------------------------------------------------------ matrix.rs */
  CASE("matrix_multiply_two_matrices") { /* matrix.rs:373 */
    double a[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 8, 7, 6, 5, 4, 3, 2};
    double b[] = {-2, 1, 2, 3, 3, 2, 1, -1, 4, 3, 6, 5, 1, 2, 7, 8};
    double e[] = {20, 22, 50, 48, 44, 54, 114, 108, 40, 58, 110, 102, 16, 26, 46, 42};
    omat A = M4(a), B = M4(b), E = M4(e), C = om_mul(&A, &B);
    CHECK(om_eq(&C, &E));
  }
  CASE("matrix_multiply_point_vector") { /* matrix.rs:397,407 */
    double a[] = {1, 2, 3, 4, 2, 4, 4, 2, 8, 6, 4, 1, 0, 0, 0, 1};
    omat A = M4(a);
    CHECK_T3(om_mul_point(&A, or_t3(1, 2, 3)), 18, 24, 33);
    CHECK_T3(om_mul_vector(&A, or_t3(1, 2, 3)), 14, 22, 32);
  }
  CASE("matrix_determinant_4x4") { /* matrix.rs:514 */
    double a[] = {-2, -8, 3, 5, -3, 1, 7, 3, 1, 2, -9, 6, -6, 7, 7, -9};
    omat A = M4(a);
    CHECK_EQ(om_cofactor(&A, 0, 0), 690.0); CHECK_EQ(om_cofactor(&A, 0, 1), 447.0);
    CHECK_EQ(om_cofactor(&A, 0, 2), 210.0); CHECK_EQ(om_cofactor(&A, 0, 3), 51.0);
    CHECK_EQ(om_determinant(&A), -4071.0);
  }
  CASE("matrix_determinant_3x3_cofactors") { /* matrix.rs:477-505 */
    double a[] = {1, 2, 6, -5, 8, -4, 2, 6, 4};
    omat A = om_from(3, 3, a);
    CHECK_EQ(om_cofactor(&A, 0, 0), 56.0); CHECK_EQ(om_cofactor(&A, 0, 1), 12.0);
    CHECK_EQ(om_cofactor(&A, 0, 2), -46.0); CHECK_EQ(om_determinant(&A), -196.0);
    double b[] = {3, 5, 0, 2, -1, -7, 6, -1, 5};
    omat B = om_from(3, 3, b);
    CHECK_EQ(om_minor(&B, 1, 0), 25.0); CHECK_EQ(om_cofactor(&B, 1, 0), -25.0);
    CHECK_EQ(om_minor(&B, 0, 0), -12.0); CHECK_EQ(om_cofactor(&B, 0, 0), -12.0);
  }
  CASE("matrix_invertible_and_not") { /* matrix.rs:533,551 */
    double a[] = {6, 4, 4, 4, 5, 5, 7, 6, 4, -9, 3, -7, 9, 1, 7, -6};
    double b[] = {-4, 2, -2, -3, 9, 6, 2, 6, 0, -5, 1, -5, 0, 0, 0, 0};
    omat A = M4(a), B = M4(b), X;
    CHECK_EQ(om_determinant(&A), -2120.0); CHECK(om_is_invertible(&A));
    CHECK_EQ(om_determinant(&B), 0.0); CHECK(!om_is_invertible(&B));
    CHECK(om_inverse(&B, &X) == RT_ERR_NOT_INVERTIBLE);
  }
  CASE("matrix_inverse_1") { /* matrix.rs:569 */
    double a[] = {-5, 2, 6, -8, 1, -5, 1, 8, 7, 7, -6, -7, 1, -3, 7, 4};
    double e[] = {0.21805, 0.45113, 0.24060, -0.04511, -0.80827, -1.45677, -0.44361, 0.52068,
                  -0.07895, -0.22368, -0.05263, 0.19737, -0.52256, -0.81391, -0.30075, 0.30639};
    omat A = M4(a), B, E = M4(e);
    CHECK(om_inverse(&A, &B) == RT_OK);
    CHECK_EQ(om_determinant(&A), 532.0);
    CHECK_EQ(om_cofactor(&A, 2, 3), -160.0); CHECK_EQ(om_at(&B, 3, 2), -160.0 / 532.0);
    CHECK_EQ(om_cofactor(&A, 3, 2), 105.0); CHECK_EQ(om_at(&B, 2, 3), 105.0 / 532.0);
    CHECK(om_eq(&B, &E));
  }
  CASE("matrix_inverse_3") { /* matrix.rs:606 */
    double a[] = {9, 3, 0, 9, -5, -2, -6, -3, -4, 9, 6, 4, -7, 6, 6, 2};
    double e[] = {-0.04074, -0.07778, 0.14444, -0.22222, -0.07778, 0.03333, 0.36667, -0.33333,
                  -0.02901, -0.14630, -0.10926, 0.12963, 0.17778, 0.06667, -0.26667, 0.33333};
    omat A = M4(a), B, E = M4(e);
    om_inverse(&A, &B);
    CHECK(om_eq(&B, &E));
  }
  CASE("matrix_product_by_inverse") { /* matrix.rs:630 */
    double a[] = {3, -9, 7, 3, 3, -8, 2, -9, -4, 4, 4, 1, -6, 5, -1, 1};
    double b[] = {8, 2, 2, 2, 3, -1, 7, 0, 7, 0, 5, 4, 6, -2, 0, 5};
    omat A = M4(a), B = M4(b), C = om_mul(&A, &B), Bi;
    om_inverse(&B, &Bi);
    omat D = om_mul(&C, &Bi);
    CHECK(om_eq(&D, &A));
  }
  CASE("transform_chain") { /* transform.rs:270; matrix.rs:656 */
    omat a = or_rotation_x(PI / 2.0), b = or_scaling(5, 5, 5), c = or_translation(10, 5, 7);
    omat cb = om_mul(&c, &b), t = om_mul(&cb, &a);
    CHECK_T3(om_mul_point(&t, or_t3(1, 0, 1)), 15, 0, 7);
  }
  CASE("view_transform_default_and_axes") { /* transform.rs:281,290,299 */
    omat t = or_view_transform(or_t3(0, 0, 0), or_t3(0, 0, -1), or_t3(0, 1, 0));
    omat id = om_identity(4);
    CHECK(om_eq(&t, &id));
    t = or_view_transform(or_t3(0, 0, 0), or_t3(0, 0, 1), or_t3(0, 1, 0));
    omat s = or_scaling(-1, 1, -1);
    CHECK(om_eq(&t, &s));
    t = or_view_transform(or_t3(0, 0, 8), or_t3(0, 0, 0), or_t3(0, 1, 0));
    omat tr = or_translation(0, 0, -8);
    CHECK(om_eq(&t, &tr));
  }
  CASE("view_transform_arbitrary") { /* transform.rs:308 */
    omat t = or_view_transform(or_t3(1, 3, 2), or_t3(4, -2, 8), or_t3(1, 1, 0));
    double e[] = {-0.50709, 0.50709, 0.67612, -2.36643, 0.76772, 0.60609, 0.12122, -2.82843,
                  -0.35857, 0.59761, -0.71714, 0.0, 0.0, 0.0, 0.0, 1.0};
    omat E = M4(e);
    CHECK(om_eq(&t, &E));
  }

  /* ----------------------------------------------------- shapes / geometry */
  CASE("sphere_intersections") { /* sphere.rs:91-159 */
    oshape s = or_sphere_default();
    double t[OR_MAX_LOCAL_XS];
    CHECK(count_intersect(&s, R(0, 0, -5, 0, 0, 1), t) == 2); CHECK_EQ(t[0], 4.0); CHECK_EQ(t[1], 6.0);
    CHECK(count_intersect(&s, R(0, 1, -5, 0, 0, 1), t) == 2); CHECK_EQ(t[0], 5.0); CHECK_EQ(t[1], 5.0);
    CHECK(count_intersect(&s, R(0, 2, -5, 0, 0, 1), t) == 0);
    CHECK(count_intersect(&s, R(0, 0, 0, 0, 0, 1), t) == 2); CHECK_EQ(t[0], -1.0); CHECK_EQ(t[1], 1.0);
    CHECK(count_intersect(&s, R(0, 0, 5, 0, 0, 1), t) == 2); CHECK_EQ(t[0], -6.0); CHECK_EQ(t[1], -4.0);
    oshape s2 = or_sphere_default();
    set_tf(&s2, or_scaling(2, 2, 2));
    CHECK(count_intersect(&s2, R(0, 0, -5, 0, 0, 1), t) == 2); CHECK_EQ(t[0], 3.0); CHECK_EQ(t[1], 7.0);
    oshape s3 = or_sphere_default();
    set_tf(&s3, or_translation(5, 0, 0));
    CHECK(count_intersect(&s3, R(0, 0, -5, 0, 0, 1), t) == 0);
  }
  CASE("sphere_normals") { /* sphere.rs:161-237 */
    oshape s = or_sphere_default();
    CHECK_T3(or_normal_at(&s, or_t3(1, 0, 0)), 1, 0, 0);
    CHECK_T3(or_normal_at(&s, or_t3(0, 1, 0)), 0, 1, 0);
    CHECK_T3(or_normal_at(&s, or_t3(0, 0, 1)), 0, 0, 1);
    ot3 n = or_normal_at(&s, or_t3(S3, S3, S3));
    CHECK_T3(n, S3, S3, S3);
    CHECK(or_t3_eq(n, or_normalize(n)));
    oshape s2 = or_sphere_default();
    set_tf(&s2, or_translation(0, 1, 0));
    CHECK_T3(or_normal_at(&s2, or_t3(0.0, 1.70711, -0.70710678118654752)), 0.0, 0.70710678118654752, -0.70710678118654752);
    oshape s3 = or_sphere_default();
    omat sc = or_scaling(1.0, 0.5, 1.0), rz = or_rotation_z(PI / 5.0);
    set_tf(&s3, om_mul(&sc, &rz));
    CHECK_T3(or_normal_at(&s3, or_t3(0.0, S2, -S2)), 0.0, 0.97014, -0.24254);
  }
  CASE("plane_intersections_normal") { /* plane.rs:73-118 */
    oshape p = or_plane_default();
    CHECK_T3(or_normal_at(&p, or_t3(0, 0, 0)), 0, 1, 0);
    CHECK_T3(or_normal_at(&p, or_t3(10, 0, -10)), 0, 1, 0);
    double t[OR_MAX_LOCAL_XS];
    oray r = R(0, 10, 0, 0, 0, 1);
    CHECK(or_local_intersect(&p, &r, t) == 0);
    r = R(0, 0, 0, 0, 0, 1);
    CHECK(or_local_intersect(&p, &r, t) == 0);
    r = R(0, 1, 0, 0, -1, 0);
    CHECK(or_local_intersect(&p, &r, t) == 1); CHECK_EQ(t[0], 1.0);
    r = R(0, -1, 0, 0, 1, 0);
    CHECK(or_local_intersect(&p, &r, t) == 1); CHECK_EQ(t[0], 1.0);
  }
  CASE("object_space_ray") { /* test_shape.rs:98-120 via Ray::transform */
    oshape s = or_sphere_default();
    set_tf(&s, or_scaling(2, 2, 2));
    ot3 o = om_mul_point(&s.inverse, or_t3(0, 0, -5)), d = om_mul_vector(&s.inverse, or_t3(0, 0, 1));
    CHECK_T3(o, 0, 0, -2.5); CHECK_T3(d, 0, 0, 0.5);
    set_tf(&s, or_translation(5, 0, 0));
    o = om_mul_point(&s.inverse, or_t3(0, 0, -5)); d = om_mul_vector(&s.inverse, or_t3(0, 0, 1));
    CHECK_T3(o, -5, 0, -5); CHECK_T3(d, 0, 0, 1);
  }
  CASE("hit_rules") { /* intersection.rs:194-235 */
    oxs a[] = {{1.0, 0}, {2.0, 0}};
    or_sort_intersections(a, 2); CHECK(or_hit(a, 2) == 0 && a[0].t == 1.0);
    oxs b[] = {{-1.0, 0}, {1.0, 0}};
    or_sort_intersections(b, 2); CHECK(or_hit(b, 2) >= 0 && b[or_hit(b, 2)].t == 1.0);
    oxs c[] = {{-2.0, 0}, {-1.0, 0}};
    or_sort_intersections(c, 2); CHECK(or_hit(c, 2) == -1);
    oxs d[] = {{5.0, 0}, {7.0, 0}, {-3.0, 0}, {2.0, 0}};
    or_sort_intersections(d, 4); CHECK(d[or_hit(d, 4)].t == 2.0);
  }

  /* world fixtures */
  oworld w;
  or_world_default(&w);

  CASE("computations_outside_inside") { /* intersection.rs:237-269 */
    oworld ws; or_world_init(&ws);
    oshape s = or_sphere_default();
    or_world_add_object(&ws, &s);
    oray r = R(0, 0, -5, 0, 0, 1);
    oxs i = {4.0, 0};
    ocomps c = or_prepare_computations(&ws, &i, &r, &i, 1);
    CHECK_EQ(c.t, 4.0); CHECK_T3(c.point, 0, 0, -1); CHECK_T3(c.eyev, 0, 0, -1);
    CHECK_T3(c.normalv, 0, 0, -1); CHECK(c.inside == 0);
    r = R(0, 0, 0, 0, 0, 1);
    oxs i2 = {1.0, 0};
    c = or_prepare_computations(&ws, &i2, &r, &i2, 1);
    CHECK_T3(c.point, 0, 0, 1); CHECK_T3(c.eyev, 0, 0, -1); CHECK(c.inside == 1); CHECK_T3(c.normalv, 0, 0, -1);
    or_world_free(&ws);
  }
  CASE("computations_over_under_reflectv") { /* intersection.rs:272-295,337-346 */
    oworld ws; or_world_init(&ws);
    oshape s = or_sphere_default();
    set_tf(&s, or_translation(0, 0, 1));
    or_world_add_object(&ws, &s);
    oray r = R(0, 0, -5, 0, 0, 1);
    oxs i = {5.0, 0};
    ocomps c = or_prepare_computations(&ws, &i, &r, &i, 1);
    CHECK(c.over_point.z < -OR_EPSILON / 2.0); CHECK(c.point.z > c.over_point.z);
    CHECK(c.under_point.z > OR_EPSILON / 2.0); CHECK(c.point.z < c.under_point.z);
    oworld wp; or_world_init(&wp);
    oshape p = or_plane_default();
    or_world_add_object(&wp, &p);
    r = R(0, 1, -1, 0.0, -S2, S2);
    oxs ip = {sqrt(2.0), 0};
    c = or_prepare_computations(&wp, &ip, &r, &ip, 1);
    CHECK_T3(c.reflectv, 0.0, S2, S2);
    or_world_free(&ws); or_world_free(&wp);
  }
  CASE("n1_n2_at_various_intersections") { /* intersection.rs:297-335 */
    oworld wg; or_world_init(&wg);
    oshape a = or_sphere_glass(); set_tf(&a, or_scaling(2, 2, 2)); a.material.refractive_index = 1.5;
    oshape b = or_sphere_glass(); set_tf(&b, or_translation(0.0, 0.0, -0.25)); b.material.refractive_index = 2.0;
    oshape c = or_sphere_glass(); set_tf(&c, or_translation(0.0, 0.0, 0.25)); c.material.refractive_index = 2.5;
    or_world_add_object(&wg, &a); or_world_add_object(&wg, &b); or_world_add_object(&wg, &c);
    oray r = R(0, 0, -4, 0, 0, 1);
    oxs xs[] = {{2.0, 0}, {2.75, 1}, {3.25, 2}, {4.75, 1}, {5.25, 2}, {6.0, 0}};
    or_sort_intersections(xs, 6);
    double ex[6][2] = {{1.0, 1.5}, {1.5, 2.0}, {2.0, 2.5}, {2.5, 2.5}, {2.5, 1.5}, {1.5, 1.0}};
    for (int k = 0; k < 6; ++k) {
      ocomps cc = or_prepare_computations(&wg, &xs[k], &r, xs, 6);
      CHECK_EQ(cc.n1, ex[k][0]); CHECK_EQ(cc.n2, ex[k][1]);
    }
    or_world_free(&wg);
  }
  CASE("schlick_cases") { /* intersection.rs:348-390 */
    oworld wg; or_world_init(&wg);
    oshape g = or_sphere_glass();
    or_world_add_object(&wg, &g);
    oray r = R(0.0, 0.0, S2, 0, 1, 0);
    oxs xs[] = {{-S2, 0}, {S2, 0}};
    ocomps c = or_prepare_computations(&wg, &xs[1], &r, xs, 2);
    CHECK_EQ(or_schlick(&c), 1.0);
    r = R(0, 0, 0, 0, 1, 0);
    oxs xs2[] = {{-1.0, 0}, {1.0, 0}};
    or_sort_intersections(xs2, 2);
    c = or_prepare_computations(&wg, &xs2[1], &r, xs2, 2);
    CHECK_EQ(or_schlick(&c), 0.04);
    r = R(0.0, 0.99, -2.0, 0, 0, 1);
    oxs xs3[] = {{1.8589, 0}};
    c = or_prepare_computations(&wg, &xs3[0], &r, xs3, 1);
    CHECK_EQ(or_schlick(&c), 0.48873);
    or_world_free(&wg);
  }
  CASE("shadow_hit_skips_no_shadow") { /* intersection.rs:404-418 */
    oworld ws; or_world_init(&ws);
    oshape s1 = or_sphere_default(); s1.shadow = 0;
    oshape s2 = or_sphere_default();
    or_world_add_object(&ws, &s1); or_world_add_object(&ws, &s2);
    /* shadow_hit over [1.0 s1, 2.0 s1, 1.0 s2, 2.0 s2]: expect the (1.0, s2) entry */
    oray r = R(-10, 0, -10, 0, 0, 1); /* unused geometry; exercise via is_shadowed below */
    (void)r;
    olight l = {or_t3(0, 0, -10), or_t3(1, 1, 1)};
    /* point at origin inside both spheres: only s2 may shadow */
    CHECK(or_is_shadowed(&ws, or_t3(0, 0, 5), &l, NULL) == 1);
    ws.objects[1].shadow = 0;
    CHECK(or_is_shadowed(&ws, or_t3(0, 0, 5), &l, NULL) == 0);
    or_world_free(&ws);
  }

  /* ------------------------------------------------------------ material.rs */
  CASE("lighting_cases") { /* material.rs:105-202 */
    omaterial m = or_material_default();
    oshape s = or_sphere_default();
    olight l = {or_t3(0, 0, -10), or_t3(1, 1, 1)};
    CHECK_T3(or_lighting(&m, &s, &l, or_t3(0, 0, 0), or_t3(0, 0, -1), or_t3(0, 0, -1), 0), 1.9, 1.9, 1.9);
    CHECK_T3(or_lighting(&m, &s, &l, or_t3(0, 0, 0), or_t3(0.0, S2, -S2), or_t3(0, 0, -1), 0), 1.0, 1.0, 1.0);
    olight l2 = {or_t3(0, 10, -10), or_t3(1, 1, 1)};
    CHECK_T3(or_lighting(&m, &s, &l2, or_t3(0, 0, 0), or_t3(0, 0, -1), or_t3(0, 0, -1), 0), 0.7364, 0.7364, 0.7364);
    CHECK_T3(or_lighting(&m, &s, &l2, or_t3(0, 0, 0), or_t3(0.0, -S2, -S2), or_t3(0, 0, -1), 0), 1.6364, 1.6364, 1.6364);
    olight l3 = {or_t3(0, 0, 10), or_t3(1, 1, 1)};
    CHECK_T3(or_lighting(&m, &s, &l3, or_t3(0, 0, 0), or_t3(0, 0, -1), or_t3(0, 0, -1), 0), 0.1, 0.1, 0.1);
    CHECK_T3(or_lighting(&m, &s, &l, or_t3(0, 0, 0), or_t3(0, 0, -1), or_t3(0, 0, -1), 1), 0.1, 0.1, 0.1);
  }
  CASE("lighting_with_pattern") { /* material.rs:205-231 */
    omaterial m = or_material_default();
    m.has_pattern = 1;
    m.pattern = or_pattern(RT_PATTERN_STRIPE, or_t3(1, 1, 1), or_t3(0, 0, 0));
    m.ambient = 1.0; m.diffuse = 0.0; m.specular = 0.0;
    oshape s = or_sphere_default();
    olight l = {or_t3(0, 0, -10), or_t3(1, 1, 1)};
    CHECK_T3(or_lighting(&m, &s, &l, or_t3(0.9, 0, 0), or_t3(0, 0, -1), or_t3(0, 0, -1), 0), 1, 1, 1);
    CHECK_T3(or_lighting(&m, &s, &l, or_t3(1.1, 0, 0), or_t3(0, 0, -1), or_t3(0, 0, -1), 0), 0, 0, 0);
  }

  /* ---------------------------------------------------------------- pattern */
  CASE("stripe_pattern") { /* stripe.rs:44-117 */
    opattern p = or_pattern(RT_PATTERN_STRIPE, or_t3(1, 1, 1), or_t3(0, 0, 0));
    double xs[] = {0, 0.9, 1, -0.1, -1, -1.1};
    double ex[] = {1, 1, 0, 0, 0, 1};
    for (int k = 0; k < 6; ++k) CHECK_EQ(or_pattern_color_at(&p, or_t3(xs[k], 0, 0)).x, ex[k]);
    for (int k = 0; k < 3; ++k) {
      CHECK_EQ(or_pattern_color_at(&p, or_t3(0, k, 0)).x, 1.0);
      CHECK_EQ(or_pattern_color_at(&p, or_t3(0, 0, k)).x, 1.0);
    }
    oshape o = or_sphere_default(); set_tf(&o, or_scaling(2, 2, 2));
    CHECK_T3(or_pattern_color_at_shape(&p, &o, or_t3(1.5, 0, 0)), 1, 1, 1);
    oshape o2 = or_sphere_default();
    opattern p2 = p; omat sc = or_scaling(2, 2, 2); or_pattern_set_transform(&p2, &sc);
    CHECK_T3(or_pattern_color_at_shape(&p2, &o2, or_t3(1.5, 0, 0)), 1, 1, 1);
    opattern p3 = p; omat tr = or_translation(0.5, 0, 0); or_pattern_set_transform(&p3, &tr);
    CHECK_T3(or_pattern_color_at_shape(&p3, &o, or_t3(2.5, 0, 0)), 1, 1, 1);
  }
  CASE("gradient_ring_checkers") { /* gradient.rs:29-46, ring.rs:32-40, checkers.rs:32-59 */
    opattern g = or_pattern(RT_PATTERN_GRADIENT, or_t3(1, 1, 1), or_t3(0, 0, 0));
    CHECK_T3(or_pattern_color_at(&g, or_t3(0, 0, 0)), 1, 1, 1);
    CHECK_T3(or_pattern_color_at(&g, or_t3(0.25, 0, 0)), 0.75, 0.75, 0.75);
    CHECK_T3(or_pattern_color_at(&g, or_t3(0.5, 0, 0)), 0.5, 0.5, 0.5);
    CHECK_T3(or_pattern_color_at(&g, or_t3(0.75, 0, 0)), 0.25, 0.25, 0.25);
    opattern r = or_pattern(RT_PATTERN_RING, or_t3(1, 1, 1), or_t3(0, 0, 0));
    CHECK_T3(or_pattern_color_at(&r, or_t3(0, 0, 0)), 1, 1, 1);
    CHECK_T3(or_pattern_color_at(&r, or_t3(1, 0, 0)), 0, 0, 0);
    CHECK_T3(or_pattern_color_at(&r, or_t3(0, 0, 1)), 0, 0, 0);
    CHECK_T3(or_pattern_color_at(&r, or_t3(0.708, 0, 0.708)), 0, 0, 0);
    opattern c = or_pattern(RT_PATTERN_CHECKERS, or_t3(1, 1, 1), or_t3(0, 0, 0));
    CHECK_T3(or_pattern_color_at(&c, or_t3(0, 0, 0)), 1, 1, 1);
    CHECK_T3(or_pattern_color_at(&c, or_t3(0.99, 0, 0)), 1, 1, 1);
    CHECK_T3(or_pattern_color_at(&c, or_t3(1.01, 0, 0)), 0, 0, 0);
    CHECK_T3(or_pattern_color_at(&c, or_t3(0, 0.99, 0)), 1, 1, 1);
    CHECK_T3(or_pattern_color_at(&c, or_t3(0, 1.01, 0)), 0, 0, 0);
    CHECK_T3(or_pattern_color_at(&c, or_t3(0, 0, 0.99)), 1, 1, 1);
    CHECK_T3(or_pattern_color_at(&c, or_t3(0, 0, 1.01)), 0, 0, 0);
  }
  CASE("test_pattern_transforms") { /* test_pattern.rs:39-68 */
    opattern p = or_pattern(RT_PATTERN_TEST, or_t3(0, 0, 0), or_t3(0, 0, 0));
    oshape o = or_sphere_default(); set_tf(&o, or_scaling(2, 2, 2));
    CHECK_T3(or_pattern_color_at_shape(&p, &o, or_t3(2, 3, 4)), 1.0, 1.5, 2.0);
    oshape o2 = or_sphere_default();
    opattern p2 = p; omat sc = or_scaling(2, 2, 2); or_pattern_set_transform(&p2, &sc);
    CHECK_T3(or_pattern_color_at_shape(&p2, &o2, or_t3(2, 3, 4)), 1.0, 1.5, 2.0);
    opattern p3 = p; omat tr = or_translation(0.5, 1.0, 1.5); or_pattern_set_transform(&p3, &tr);
    CHECK_T3(or_pattern_color_at_shape(&p3, &o, or_t3(2.5, 3.0, 3.5)), 0.75, 0.5, 0.25);
  }

  /* ---------------------------------------------------------------- world.rs */
  CASE("world_intersect") { /* world.rs:185-195 */
    oray r = R(0, 0, -5, 0, 0, 1);
    int n;
    oxs* xs = or_world_intersect(&w, &r, &n, NULL);
    CHECK(n == 4);
    if (n == 4) { CHECK_EQ(xs[0].t, 4.0); CHECK_EQ(xs[1].t, 4.5); CHECK_EQ(xs[2].t, 5.5); CHECK_EQ(xs[3].t, 6.0); }
    free(xs);
  }
  CASE("shade_intersection") { /* world.rs:197-206 */
    oray r = R(0, 0, -5, 0, 0, 1);
    oxs i = {4.0, 0};
    ocomps c = or_prepare_computations(&w, &i, &r, &i, 1);
    CHECK_T3(or_shade_hit(&w, &c, 5, NULL), 0.38066, 0.47583, 0.2855);
  }
  CASE("shade_intersection_inside") { /* world.rs:208-218 */
    oworld w2; or_world_default(&w2);
    w2.lights[0].position = or_t3(0.0, 0.25, 0.0);
    oray r = R(0, 0, 0, 0, 0, 1);
    oxs i = {0.5, 1};
    ocomps c = or_prepare_computations(&w2, &i, &r, &i, 1);
    CHECK_T3(or_shade_hit(&w2, &c, 5, NULL), 0.90498, 0.90498, 0.90498);
    or_world_free(&w2);
  }
  CASE("color_at_miss_hit") { /* world.rs:220-234 */
    oray r = R(0, 0, -5, 0, 1, 0);
    CHECK_T3(or_color_at(&w, &r, 5, NULL), 0, 0, 0);
    r = R(0, 0, -5, 0, 0, 1);
    CHECK_T3(or_color_at(&w, &r, 5, NULL), 0.38066, 0.47583, 0.2855);
  }
  CASE("is_shadowed_cases") { /* world.rs:248-274 */
    CHECK(or_is_shadowed(&w, or_t3(0, 10, 0), &w.lights[0], NULL) == 0);
    CHECK(or_is_shadowed(&w, or_t3(10, -10, 10), &w.lights[0], NULL) == 1);
    CHECK(or_is_shadowed(&w, or_t3(-20, 20, -20), &w.lights[0], NULL) == 0);
    CHECK(or_is_shadowed(&w, or_t3(-2, 2, -2), &w.lights[0], NULL) == 0);
  }
  CASE("shade_hit_in_shadow") { /* world.rs:276-293 */
    oworld w2; or_world_init(&w2);
    or_world_add_light(&w2, or_t3(0, 0, -10), or_t3(1, 1, 1));
    oshape s1 = or_sphere_default(), s2 = or_sphere_default();
    set_tf(&s2, or_translation(0, 0, 10));
    or_world_add_object(&w2, &s1); or_world_add_object(&w2, &s2);
    oray r = R(0, 0, 5, 0, 0, 1);
    oxs i = {4.0, 1};
    ocomps c = or_prepare_computations(&w2, &i, &r, &i, 1);
    CHECK_T3(or_shade_hit(&w2, &c, 5, NULL), 0.1, 0.1, 0.1);
    or_world_free(&w2);
  }
  CASE("reflected_color_non_reflective") { /* world.rs:295-309 */
    oworld w2; or_world_default(&w2);
    w2.objects[1].material.ambient = 1.0;
    oray r = R(0, 0, 0, 0, 0, 1);
    oxs i = {1.0, 1};
    ocomps c = or_prepare_computations(&w2, &i, &r, &i, 1);
    CHECK_T3(or_reflected_color(&w2, &c, 5, NULL), 0, 0, 0);
    or_world_free(&w2);
  }
  /* world.rs:311-347,368-383: the reflective plane fixtures */
  {
    oworld w2; or_world_default(&w2);
    oshape pl = or_plane_default();
    pl.material.reflective = 0.5;
    set_tf(&pl, or_translation(0, -1, 0));
    or_world_add_object(&w2, &pl);
    oray r = R(0, 0, -3, 0.0, -S2, S2);
    oxs i = {sqrt(2.0), 2};
    ocomps c = or_prepare_computations(&w2, &i, &r, &i, 1);
    CASE("reflected_color_reflective") { CHECK_T3(or_reflected_color(&w2, &c, 5, NULL), 0.19033, 0.23791, 0.14274); }
    CASE("shade_hit_reflective") { CHECK_T3(or_shade_hit(&w2, &c, 5, NULL), 0.87676, 0.92435, 0.82918); }
    CASE("reflected_color_max_depth") {
      oxs i0 = {sqrt(2.0), 0};
      ocomps c0 = or_prepare_computations(&w2, &i0, &r, &i0, 1);
      CHECK_T3(or_reflected_color(&w2, &c0, 0, NULL), 0, 0, 0);
    }
    or_world_free(&w2);
  }
  CASE("mutually_reflective_terminates") { /* world.rs:349-366 */
    oworld w2; or_world_init(&w2);
    or_world_add_light(&w2, or_t3(0, 0, 0), or_t3(1, 1, 1));
    oshape lo = or_plane_default(); lo.material.reflective = 1.0; set_tf(&lo, or_translation(0, -1, 0));
    oshape up = or_plane_default(); up.material.reflective = 1.0; set_tf(&up, or_translation(0, 1, 0));
    or_world_add_object(&w2, &lo); or_world_add_object(&w2, &up);
    oray r = R(0, 0, 0, 0, 1, 0);
    rt_stats st; memset(&st, 0, sizeof st);
    or_color_at(&w2, &r, 5, &st);
    CHECK(st.rays_primary + st.rays_reflect == 6);
    or_world_free(&w2);
  }
  CASE("refracted_color_opaque") { /* world.rs:385-397 */
    oray r = R(0, 0, -5, 0, 0, 1);
    oxs xs[] = {{4.0, 0}, {6.0, 0}};
    ocomps c = or_prepare_computations(&w, &xs[0], &r, xs, 2);
    CHECK_T3(or_refracted_color(&w, &c, 5, NULL), 0, 0, 0);
  }
  CASE("refracted_color_max_depth") { /* world.rs:399-416 */
    oworld w2; or_world_default(&w2);
    w2.objects[0].material.transparency = 1.0; w2.objects[0].material.refractive_index = 1.5;
    oray r = R(0, 0, 5, 0, 0, 1);
    oxs xs[] = {{4.0, 0}, {6.0, 0}};
    ocomps c = or_prepare_computations(&w2, &xs[0], &r, xs, 2);
    CHECK_T3(or_refracted_color(&w2, &c, 0, NULL), 0, 0, 0);
    or_world_free(&w2);
  }
  CASE("refracted_color_total_internal_reflection") { /* world.rs:418-438 */
    oworld w2; or_world_default(&w2);
    w2.objects[0].material.transparency = 1.0; w2.objects[0].material.refractive_index = 1.5;
    oray r = R(0.0, 0.0, S2, 0, 1, 0);
    oxs xs[] = {{-S2, 0}, {S2, 0}};
    ocomps c = or_prepare_computations(&w2, &xs[1], &r, xs, 2);
    CHECK_T3(or_refracted_color(&w2, &c, 5, NULL), 0, 0, 0);
    or_world_free(&w2);
  }
  CASE("refracted_color_with_refracted_ray") { /* world.rs:440-463 */
    oworld w2; or_world_default(&w2);
    w2.objects[0].material.ambient = 1.0;
    w2.objects[0].material.has_pattern = 1;
    w2.objects[0].material.pattern = or_pattern(RT_PATTERN_TEST, or_t3(0, 0, 0), or_t3(0, 0, 0));
    w2.objects[1].material.transparency = 1.0; w2.objects[1].material.refractive_index = 1.5;
    oray r = R(0.0, 0.0, 0.1, 0, 1, 0);
    oxs xs[] = {{-0.9899, 0}, {-0.4899, 1}, {0.4899, 1}, {0.9899, 0}};
    or_sort_intersections(xs, 4);
    ocomps c = or_prepare_computations(&w2, &xs[2], &r, xs, 4);
    CHECK_T3(or_refracted_color(&w2, &c, 5, NULL), 0.0, 0.99887, 0.04722);
    or_world_free(&w2);
  }
  CASE("shade_hit_transparent") { /* world.rs:465-491 */
    oworld w2; or_world_default(&w2);
    oshape floor = or_plane_default(); set_tf(&floor, or_translation(0, -1, 0));
    floor.material.transparency = 0.5; floor.material.refractive_index = 1.5;
    or_world_add_object(&w2, &floor);
    oshape ball = or_sphere_default(); ball.material.color = or_t3(1.0, 0.0, 0.0); ball.material.ambient = 0.5;
    set_tf(&ball, or_translation(0.0, -3.5, -0.5));
    or_world_add_object(&w2, &ball);
    oray r = R(0, 0, -3, 0.0, -S2, S2);
    oxs xs[] = {{sqrt(2.0), 2}};
    ocomps c = or_prepare_computations(&w2, &xs[0], &r, xs, 1);
    CHECK_T3(or_shade_hit(&w2, &c, 5, NULL), 0.93642, 0.68642, 0.68642);
    or_world_free(&w2);
  }
  CASE("shade_hit_schlick") { /* world.rs:493-520 */
    oworld w2; or_world_default(&w2);
    oshape floor = or_plane_default(); set_tf(&floor, or_translation(0, -1, 0));
    floor.material.reflective = 0.5; floor.material.transparency = 0.5; floor.material.refractive_index = 1.5;
    or_world_add_object(&w2, &floor);
    oshape ball = or_sphere_default(); ball.material.color = or_t3(1.0, 0.0, 0.0); ball.material.ambient = 0.5;
    set_tf(&ball, or_translation(0.0, -3.5, -0.5));
    or_world_add_object(&w2, &ball);
    oray r = R(0, 0, -3, 0.0, -S2, S2);
    oxs xs[] = {{sqrt(2.0), 2}};
    ocomps c = or_prepare_computations(&w2, &xs[0], &r, xs, 1);
    CHECK_T3(or_shade_hit(&w2, &c, 5, NULL), 0.93391, 0.69643, 0.69243);
    or_world_free(&w2);
  }

  /* -------------------------------------------------------------- camera.rs */
  CASE("camera_pixel_size") { /* camera.rs:287-297 */
    ocamera c;
    or_camera_new(&c, 200, 125, PI / 2.0); CHECK_EQ(c.pixel_size, 0.01);
    or_camera_new(&c, 125, 200, PI / 2.0); CHECK_EQ(c.pixel_size, 0.01);
  }
  CASE("camera_rays") { /* camera.rs:299-325 */
    ocamera c;
    or_camera_new(&c, 201, 101, PI / 2.0);
    oray r = or_ray_for_pixel(&c, 100, 50);
    CHECK_T3(r.origin, 0, 0, 0); CHECK_T3(r.direction, 0, 0, -1);
    r = or_ray_for_pixel(&c, 0, 0);
    CHECK_T3(r.origin, 0, 0, 0); CHECK_T3(r.direction, 0.66519, 0.33259, -0.66851);
    omat ry = or_rotation_y(PI / 4.0), tr = or_translation(0, -2, 5), t = om_mul(&ry, &tr);
    or_camera_set_transform(&c, &t);
    r = or_ray_for_pixel(&c, 100, 50);
    CHECK_T3(r.origin, 0, 2, -5); CHECK_T3(r.direction, S2 * 2.0 / 2.0 * 1.0, 0.0, -S2);
  }
  CASE("render_world_with_camera") { /* camera.rs:327-337 */
    ocamera c;
    or_camera_new(&c, 11, 11, PI / 2.0);
    omat vt = or_view_transform(or_t3(0, 0, -5), or_t3(0, 0, 0), or_t3(0, 1, 0));
    or_camera_set_transform(&c, &vt);
    rt_camera_desc cd;
    double* img = (double*)calloc(11 * 11 * 3, sizeof(double));
    oracle_camera_init(11, 11, PI / 2.0, vt.e, &cd);
    oracle_render_rows(&w, &cd, 5, 1, NULL, 11, 2, img, NULL);
    const double* px = img + (5 * 11 + 5) * 3;
    CHECK_T3(or_t3(px[0], px[1], px[2]), 0.38066, 0.47583, 0.2855);
    free(img);
  }

  /* ---------------------------------------------------------- image/ppm.rs */
  CASE("ppm_header_and_pixels") { /* ppm.rs:81-109 */
    double img[5 * 3 * 3];
    memset(img, 0, sizeof img);
    double* p = img + (0 * 5 + 0) * 3; p[0] = 1.5;
    p = img + (1 * 5 + 2) * 3; p[1] = 0.5;
    p = img + (2 * 5 + 4) * 3; p[0] = -0.5; p[2] = 1.0;
    char buf[512];
    size_t n = or_canvas_to_ppm(img, 5, 3, buf, sizeof buf);
    const char* expect =
        "P3\n5 3\n255\n"
        "255 0 0 0 0 0 0 0 0 0 0 0 0 0 0\n"
        "0 0 0 0 0 0 0 128 0 0 0 0 0 0 0\n"
        "0 0 0 0 0 0 0 0 0 0 0 0 0 0 255\n";
    CHECK(n == strlen(expect) && memcmp(buf, expect, n) == 0);
  }
  CASE("ppm_color_component_scaling") { /* ppm.rs:111-118 */
    CHECK(or_scale_color_component(0.0) == 0);
    CHECK(or_scale_color_component(255.0) == 255);
    CHECK(or_scale_color_component(-0.5) == 0);
    CHECK(or_scale_color_component(1.5) == 255);
    CHECK(or_scale_color_component(0.5) == 128);
    CHECK(or_scale_color_component(0.1) == 26); /* 25.5 rounds away from zero */
    CHECK(or_scale_color_component(NAN) == 0);
  }
  CASE("ppm_split_long_lines") { /* ppm.rs:127-150 */
    double img[10 * 2 * 3];
    for (int k = 0; k < 20; ++k) { img[k * 3] = 1.0; img[k * 3 + 1] = 0.8; img[k * 3 + 2] = 0.6; }
    char buf[1024];
    size_t n = or_canvas_to_ppm(img, 10, 2, buf, sizeof buf);
    const char* expect =
        "P3\n10 2\n255\n"
        "255 204 153 255 204 153 255 204 153 255 204 153 255 204 153 255 204\n"
        "153 255 204 153 255 204 153 255 204 153 255 204 153\n"
        "255 204 153 255 204 153 255 204 153 255 204 153 255 204 153 255 204\n"
        "153 255 204 153 255 204 153 255 204 153 255 204 153\n";
    CHECK(n == strlen(expect) && memcmp(buf, expect, n) == 0);
  }

  /* ------------------------------------------------ bounding_box.rs / group.rs */
  CASE("bounding_box_intersects_cube_at_origin") { /* bounding_box.rs:315-357 */
    obbox b = {or_t3(-1, -1, -1), or_t3(1, 1, 1)};
    const double tc[13][7] = {{5, 0.5, 0, -1, 0, 0, 1},  {-5, 0.5, 0, 1, 0, 0, 1}, {0.5, 5, 0, 0, -1, 0, 1},
                              {0.5, -5, 0, 0, 1, 0, 1},  {0.5, 0, 5, 0, 0, -1, 1}, {0.5, 0, -5, 0, 0, 1, 1},
                              {0, 0.5, 0, 0, 0, 1, 1},   {-2, 0, 0, 2, 4, 6, 0},   {0, -2, 0, 6, 2, 4, 0},
                              {0, 0, -2, 4, 6, 2, 0},    {2, 0, 2, 0, 0, -1, 0},   {0, 2, 2, 0, -1, 0, 0},
                              {2, 2, 0, -1, 0, 0, 0}};
    for (int i = 0; i < 13; ++i) {
      oray r = {or_t3(tc[i][0], tc[i][1], tc[i][2]), or_normalize(or_t3(tc[i][3], tc[i][4], tc[i][5]))};
      CHECK(or_bbox_intersects(&b, &r) == (int)tc[i][6]);
    }
  }
  CASE("bounding_box_intersects_non_cubic") { /* bounding_box.rs:359-401 */
    obbox b = {or_t3(5, -2, 0), or_t3(11, 4, 7)};
    const double tc[13][7] = {{15, 1, 2, -1, 0, 0, 1}, {-5, -1, 4, 1, 0, 0, 1},   {7, 6, 5, 0, -1, 0, 1},
                              {9, -5, 6, 0, 1, 0, 1},  {8, 2, 12, 0, 0, -1, 1},   {6, 0, -5, 0, 0, 1, 1},
                              {8, 1, 3.5, 0, 0, 1, 1}, {9, -1, -8, 2, 4, 6, 0},   {8, 3, -4, 6, 2, 4, 0},
                              {9, -1, -2, 4, 6, 2, 0}, {4, 0, 9, 0, 0, -1, 0},    {8, 6, -1, 0, -1, 0, 0},
                              {12, 5, 4, -1, 0, 0, 0}};
    for (int i = 0; i < 13; ++i) {
      oray r = {or_t3(tc[i][0], tc[i][1], tc[i][2]), or_normalize(or_t3(tc[i][3], tc[i][4], tc[i][5]))};
      CHECK(or_bbox_intersects(&b, &r) == (int)tc[i][6]);
    }
  }
  CASE("group_box_gates_its_children") { /* bounding_box.rs:403-441, group.rs:49-58, :263-278 */
    /* a group around a unit sphere: a ray that misses the group's box intersects no child
     * (no local_intersect call); one that meets it intersects the child */
    oworld gw;
    or_world_init(&gw);
    obbox b = {or_t3(-1, -1, -1), or_t3(1, 1, 1)};
    or_world_add_group(&gw, b, -1);
    oshape s = or_sphere_default();
    s.gate = 1;
    or_world_add_object(&gw, &s);
    rt_stats st;
    memset(&st, 0, sizeof st);
    int n = 0;
    oray miss = R(0, 0, -5, 0, 1, 0);
    free(or_world_intersect(&gw, &miss, &n, &st));
    CHECK(n == 0 && st.sphere_tests == 0);
    oray hit = R(0, 0, -5, 0, 0, 1);
    free(or_world_intersect(&gw, &hit, &n, &st));
    CHECK(n == 2 && st.sphere_tests == 1);
    /* intersect_transformed_group (group.rs:263-278): scaling(2) group, child at translation(5): the
     * child's baked transform is scaling(2) * translation(5, 0, 0); the group's box is its box */
    or_world_free(&gw);
    or_world_init(&gw);
    oshape c = or_sphere_default();
    omat sc = or_scaling(2, 2, 2), tr = or_translation(5, 0, 0), m = om_mul(&sc, &tr);
    set_tf(&c, m);
    or_world_add_group(&gw, c.bbox, -1);
    c.gate = 1;
    or_world_add_object(&gw, &c);
    oray r = R(10, 0, -10, 0, 0, 1);
    oxs* xs = or_world_intersect(&gw, &r, &n, NULL);
    CHECK(n == 2);
    free(xs);
    or_world_free(&gw);
  }

  or_world_free(&w);
  printf("KAT %d/%d\n", g_total - g_failed, g_total);
  return g_failed ? 1 : 0;
}
