// rt_layout.hpp — device-resident layout of a flattened `World` (world.rs:18-21)
// shared by the host uploader (rt_api.cpp) and the HIP kernels.
//
// HBM layout (all 64-B aligned, all read-only during a render):
//   trace records  : the per-ray hot loop reads EVERY record of its class once
//                    per ray, wave-uniformly (s_load -> SGPR operands):
//       SphereDiag  8 doubles  (64 B)  inverse = diag(s) + translation t
//       SphereGen  16 doubles (128 B)  inverse rows 0-2 (general affine)
//       PlaneRec    8 doubles  (64 B)  inverse row 1 (only y matters)
//       QuadRec    16 doubles (128 B)  Cube / Cylinder / Cone: inverse rows 0-2,
//                                      minimum, maximum, kind, closed
//     each carries `meta` = (object index << 1) | casts_shadow.
//   shade records  : ShadeRec per object index (AoS, 64 doubles = 512 B),
//                    gathered per lane only at a hit.
//   lights         : 6 doubles each (position, intensity), wave-uniform.
#pragma once
#include <stdint.h>
#include <cmath>

namespace rtamd {

constexpr double kEpsilon = 0.00001;  // raytracer/src/lib.rs:18

struct alignas(64) SphereDiag {  // translation . axis scaling (e.g. all C3/C5 spheres)
  double s[3];                   // inverse diagonal m00, m11, m22
  double t[3];                   // inverse translation m03, m13, m23
  int64_t meta;
  int64_t pad;
};
// `gate`: 0, or 1 + the innermost Group the shape belongs to (GroupRec): the
// shape is tested only by rays that meet the bounding box of that group and of
// every group enclosing it (Group::intersect, group.rs:49-58; group_gate).
// Shapes inside groups are always one of these three records.
struct alignas(64) SphereGen {  // any invertible affine transform
  double m[12];                 // inverse rows 0..2
  int64_t meta;
  int32_t gate, pad0;
  int64_t pad[2];
};
struct alignas(64) PlaneRec {
  double m[4];  // inverse row 1: m10 m11 m12 m13
  int64_t meta;
  int32_t gate, pad0;
  int64_t pad[2];
};
struct alignas(64) QuadRec {  // cube.rs / cylinder.rs / cone.rs
  double m[12];  // inverse rows 0..2
  double minimum, maximum;
  int32_t kind, closed;
  int32_t meta, gate;
};
// A Group's bounding box as the reference's Group::intersect tests it
// (BaseShape::bounding_box of the group, bounding_box.rs:95-136), and 1 + the
// group enclosing it (0: a top-level group of World::objects).
struct alignas(64) GroupRec {
  double lo[3], hi[3];
  int32_t parent, pad0;
  int64_t pad;
};
static_assert(sizeof(GroupRec) == 64, "GroupRec must stay 64 B");
static_assert(sizeof(QuadRec) == 128, "QuadRec must stay 128 B");

// Bounding-volume hierarchies (built on the host, rt_bvh.cpp): one over the
// SphereDiag records, one over the other bounded records (OtherRec: general-
// transform spheres, cubes, bounded cylinders). Binary nodes carry both
// children's boxes, so one 64-B load (one s_load_dwordx16 for a wave, four
// 16-B loads for a lane) decides both children. Boxes are binary32 rounded
// OUTWARD from the padded binary64 boxes, so culling stays conservative
// (DESIGN.md "Exact culling"). A child is an internal node index (>= 0), a
// leaf code -(1 + (first << 7 | count)) over the (reordered) record array,
// or kBvhEmpty.
struct alignas(64) BvhNode {
  float lo[2][3], hi[2][3];
  int32_t child[2];
  int32_t axis;
  uint32_t pad;
};
static_assert(sizeof(BvhNode) == 64, "BvhNode must stay 64 B");
// The same node in the pair layout the per-lane traversal reads
// (lane_trace_pair): per axis a, b[4a..4a+3] = lo[0][a], lo[1][a], hi[0][a],
// hi[1][a], so the two children's entry (or exit) planes on an axis are one
// 8-B pair, chosen by the sign of the ray's direction. Its child codes are
// 16-bit, so the traversal's LDS stack is too: a node index below 0x8000, a
// leaf 0x8000 | first << 3 | (count - 1) (first < 4095, count <= 8), 0xFFFF
// empty. A hierarchy that does not fit these codes has no pair image.
struct alignas(64) BvhPair {
  float b[12];
  int32_t child[2];
  int32_t axis;
  uint32_t pad;
};
static_assert(sizeof(BvhPair) == 64, "BvhPair must stay 64 B");
// The same hierarchy collapsed to four children per node (lane_trace_wide,
// LANE 15: the whole image in LDS): one 128-B node. Slot j's box is lo[a][j],
// hi[a][j] (one 16-B load per plane block and axis), child[j] a 16-bit code: a
// node index (< 0x8000), 0x8000 | the index of one sphere record (every leaf
// holds one record), or 0xFFFF (empty; its box is inverted, lo = +inf and hi =
// -inf, so no ray with a usable axis meets it). The boxes are the binary
// nodes' own (a collapsed node's children are its binary descendants) or,
// below a binary leaf of several records, each record's own padded box (and
// unions of them) rounded outward to binary32: every box holds what lies below
// it, so every culling decision stays exact (DESIGN.md "Exact culling").
struct alignas(128) BvhWide {
  float lo[3][4];
  float hi[3][4];
  uint16_t child[4];
  uint32_t pad[6];
};
static_assert(sizeof(BvhWide) == 128, "BvhWide must stay 128 B");
// The four-wide image read from global memory (LANE 4, with a treelet of its
// top nodes in LDS): the same nodes in 64 B, the planes rounded outward again,
// to binary16 (a coordinate past binary16's range becomes an infinite plane),
// so each box still holds what lies below it. A visit reads 56 B instead of
// 104, twice the nodes fit a cache line and the treelet, and v_fma_mix_f32
// converts each half exactly inside the slab test's FMA. The culling loses
// little: the area-weighted visit cost of C3's and C5's hierarchies grows by
// 0.3 % and 0.5 %, the record tests by 1.1 % and 2.6 % (tools/wide_sah.cpp).
// (The LDS image stays binary32: there the mixed FMAs cost more issue time
// than the halved LDS reads save, C3 closest class +3 %; from global memory
// C5 runs 4 % faster)
struct alignas(64) BvhWide16 {
  uint16_t lo[3][4];  // binary16 bit patterns
  uint16_t hi[3][4];
  uint16_t child[4];
  uint32_t pad[2];
};
static_assert(sizeof(BvhWide16) == 64, "BvhWide16 must stay 64 B");
// binary16 bits -> value (host checks and tools; the device converts in the FMA)
inline float wide_f16(uint16_t b) {
  const int e = (b >> 10) & 31, m = b & 1023;
  const float v = e == 31 ? (m ? NAN : INFINITY)
                          : e == 0 ? std::ldexp((float)m, -24) : std::ldexp((float)(1024 + m), e - 25);
  return (b & 0x8000u) ? -v : v;
}
constexpr unsigned kWideEmpty = 0xFFFFu, kWideLeaf = 0x8000u;  // BvhWide child codes: empty, leaf flag
// Line hierarchy (rt_bvh.cpp build_line_bvh, line_trace): open tubes
// (cylinder.rs with closed = false) and cones (cone.rs) with finite bounds.
// Their boxes are tested over the ray's whole line up to the current hit,
// (-inf, t_hi]: a culled record then has no root at t <= t_hi at all, so it
// neither hits nor enters `containers` (an open tube is no closed solid, so
// the [0, t_hi] argument of the other hierarchies does not cover its t < 0
// roots). A cone's a ~ 0 branch (cone.rs:102-110) pushes t = -c / 2.0 * b,
// a root anywhere on the line; every other root of a cone lies in its box. So
// the cones whose a, as the reference computes it, is below EPSILON for a ray
// are found before the traversal, cluster by cluster (cone_prepass), tested
// there, and skipped by the traversal. A cluster holds the cones whose
// direction quadratic is the same (cones equal up to position and a turn
// about their axis): with the world direction d, |d|_inf = dm and g = d^T Q d
// (Q: the six distinct entries of the symmetric 3x3 form, xx yy zz xy xz yz),
// every member i has |fl(a_i) - g| <= r dm^2 (r covers every rounding, host
// and device), so |g| - r dm^2 >= EPSILON (with a margin) rules out the whole
// cluster with one test. Members: lcone[first .. first + count) (indices
// into lrec).
struct alignas(64) ConeCluster {
  double q[6];
  double r;
  int32_t first, count;
};
static_assert(sizeof(ConeCluster) == 64, "ConeCluster must stay 64 B");

// A culled record other than a diagonal sphere: the QuadRec layout, with
// kind 0 = sphere under a general inverse (rows 0-2 in m).
typedef QuadRec OtherRec;
constexpr int32_t kBvhEmpty = (int32_t)0x80000000;
constexpr int kBvhLeafMax = 127;
constexpr int kBvhMaxDepth = 60;  // traversal stack entries per wave
constexpr int kLaneLdsDepth = 16;  // per-lane traversal: LDS stack when bvh_depth fits

// Light buffer (Haines & Greenberg 1986, made exact): per point light, a
// cube map of directions around the light (6 faces x R x R cells). Cell c of
// light l lists every shadow-casting SphereDiag record whose padded box may
// hold a point whose direction from the light falls in the cell (rt_bvh.cpp
// build_light_buffer: a conservative projection with margins far above the
// query's rounding), ordered by lb_delta[l * n_diag + idx], a binary32 lower
// bound on the distance from the light to the record's box. A shadow ray from
// o is blocked only by a sphere with a root point q on the segment
// [o, light), and every such q lies in that sphere's box in the cell of
// direction o - light (DESIGN.md "Light buffer"), so testing that cell's
// list up to delta > |light - o| answers is_shadowed exactly. Records whose
// box comes near the light are listed in every cell. The answer is valid
// while |light - o| <= lb_limit[l]; farther origins take the exhaustive loop.
//
// One 16-B record per cell holds the list's first kLbInline 16-bit indices,
// so a ray makes one dependent global load for its cell; longer lists
// continue in lb_ov[ov ..].
constexpr int kLbMaxLights = 16;
constexpr int kLbInline = 5;
struct alignas(16) LbCell {
  uint32_t w0;  // count (low 16) | idx0 (high 16)
  uint32_t w1;  // idx1 | idx2 << 16
  uint32_t w2;  // idx3 | idx4 << 16
  uint32_t ov;  // entries kLbInline.. at lb_ov[ov ..]
};
static_assert(sizeof(LbCell) == 16, "LbCell must stay 16 B");

// Intersection ordering key: (object index << 2) | position in the object's
// local_intersect list (at most 4 entries, cylinder/cone). Equal t resolve by
// this key exactly like the reference's stable sort (intersection.rs:108-116).
constexpr int kKeyShift = 2;

// What a hit on an unpatterned object reads (the inverses, the material, kind
// and pattern kind) fills the first two 128-B lines; patterns, the cylinder /
// cone bounds and the host-only shadow flag come after.
struct alignas(64) ShadeRec {
  double inv[12];   // transform_inverse rows 0..2
  double invT[9];   // transform_inverse_transpose upper 3x3 (= inv^T)
  double color[3];
  double ambient, diffuse, specular, shininess;
  double reflective, transparency, refractive_index;
  int32_t kind, pattern_kind;
  double pat_a[3], pat_b[3];
  double pat_inv[12];
  int32_t shadow, pad0;
  double minimum, maximum;  // Cylinder / Cone (local_normal_at)
  double pad1[11];
};
static_assert(__builtin_offsetof(ShadeRec, pattern_kind) < 256, "hot shading fields in the first two lines");
static_assert(sizeof(ShadeRec) == 512, "ShadeRec must stay 512 B");

struct LightRec {
  double pos[3];
  double intensity[3];
};

// Kernel-argument view of a scene (passed by value; pointers live in SGPRs).
struct DevScene {
  const SphereDiag* sph_diag;
  const SphereGen* sph_gen;
  const PlaneRec* planes;
  const ShadeRec* shade;
  const LightRec* lights;
  const QuadRec* quads;
  const BvhNode* bvh;  // nullptr when the scene has no BVH
  const BvhPair* bvh_pair;  // the same nodes in the pair layout
  int32_t n_diag, n_gen, n_planes, n_objects, n_lights;
  int32_t n_quads;
  int32_t n_bvh;
  int32_t bvh_depth;  // most far children pending on a traversal stack
  // fast path: the hierarchy over the other bounded records, and what stays
  // outside every hierarchy (tested exhaustively, with the planes)
  const BvhNode* obvh;      // nullptr when there are no culled other records
  const OtherRec* orec;     // in obvh leaf order
  int32_t n_obvh, obvh_depth, n_orec;
  // the line hierarchy (line_trace): open tubes and cones with finite bounds,
  // culled over the whole line up to the hit; the cones' a ~ 0 clusters
  const BvhNode* lbvh;          // nullptr when there are none
  const QuadRec* lrec;          // in lbvh leaf order
  const ConeCluster* lclus;     // the cones' clusters (cone_prepass)
  const int32_t* lcone;         // cluster members: indices into lrec
  const int32_t* lrec_clus;     // per line record: its cone's cluster (-1: an open tube)
  int32_t n_lbvh, n_lrec, n_lclus;
  const SphereGen* fx_gen;  // general spheres outside the hierarchies
  const QuadRec* fx_quads;  // cubes / cylinders / cones outside the hierarchies
  int32_t n_fx_gen, n_fx_quads;
  const LbCell* lb_cells;  // light buffer: n_lights * 6R^2 cells, nullptr when not built
  const uint16_t* lb_ov;
  const float* lb_delta;   // n_lights * n_diag
  const float* lb_limit;   // per light
  int32_t lb_res;          // R
  int32_t lb_n_items;
  // the sphere hierarchy collapsed to four children per node (nullptr when its
  // 16-bit codes cannot index it), and the most stack entries its traversal keeps
  const BvhWide* bvhw;
  const BvhWide16* bvhw16;  // the same nodes in binary16 (the global-memory image)
  int32_t n_bvhw, bvhw_stack;
  // per object: ShadeRec::reflective, transparency (what wf_combine_parents reads; 16 B a
  // record, so the table stays in the L2 where the 512-B shading records may not)
  const double* refl_transp;
  // per object: the index of its SphereDiag record (-1: not one), after the hierarchy's reordering,
  // | kOwnOutside when a shadow ray leaving its outside provably never meets it (rt_scene.cpp)
  const int32_t* obj_diag;
  // Groups (group.rs): the records' gates index this table (rt_scene_create_groups)
  const GroupRec* groups;
  int32_t n_groups, pad_groups;
};

constexpr int32_t kOwnOutside = 0x40000000, kOwnIndex = 0x3FFFFFFF;  // DevScene::obj_diag

struct DevCamera {
  double pixel_size, half_width, half_height;
  double inv[12];
  uint32_t hsize, vsize;
};

// Counters of one render (order = rt_stats prefix, then its ABI-3 fields).
struct DevStats {
  unsigned long long rays_primary, rays_reflect, rays_refract, rays_shadow;
  unsigned long long sphere_tests, plane_tests, sphere_disc_ge0, other_tests;
  unsigned long long rays_shadow_traced, sphere_tests_executed, box_tests_executed;
  unsigned exhaustive;  // sphere_disc_ge0 is exact (every sphere tested for every reference ray)
};

}  // namespace rtamd
