// rt_scene.cpp — rt_scene_create / rt_scene_create_groups / rt_scene_destroy:
// the reference's World (world.rs:18-21, shape/group.rs) flattened into SoA
// records in the reference's object order, the exact-culling hierarchies
// (rt_bvh.cpp), the light buffer, and one upload to the scene's device.
#include "rt_api_internal.hpp"

using namespace rtapi;

namespace {

bool is_diag_inverse(const double* inv) {
  return inv[1] == 0.0 && inv[2] == 0.0 && inv[4] == 0.0 && inv[6] == 0.0 && inv[8] == 0.0 &&
         inv[9] == 0.0;
}

bool m16_eq(const double* a, const double* b) {
  for (int i = 0; i < 16; ++i)
    if (!rt::equal(a[i], b[i])) return false;
  return true;
}
bool c3_eq(const double* a, const double* b) {
  return rt::equal(a[0], b[0]) && rt::equal(a[1], b[1]) && rt::equal(a[2], b[2]);
}

// Necessary condition for the reference's structural `Shape` equality
// (derived PartialEq of BaseShape, geometry/mod.rs:12; Material, material.rs:10;
// Pattern, pattern/mod.rs:17). The bounding box is left out, so this is a
// SUPERSET of the reference relation: "no pair passes" certifies that the
// containers walk never sees two structurally-equal objects.
bool may_be_equal(const rt_shape_desc& a, const rt_shape_desc& b) {
  if (a.kind != b.kind || (a.casts_shadow != 0) != (b.casts_shadow != 0)) return false;
  if (!m16_eq(a.transform, b.transform) || !m16_eq(a.inverse, b.inverse)) return false;
  if (!c3_eq(a.color, b.color)) return false;
  if (!(a.ambient == b.ambient && a.diffuse == b.diffuse && a.specular == b.specular &&
        a.shininess == b.shininess && a.reflective == b.reflective &&
        a.transparency == b.transparency && a.refractive_index == b.refractive_index))
    return false;
  if ((a.kind == RT_SHAPE_CYLINDER || a.kind == RT_SHAPE_CONE) &&
      !(a.minimum == b.minimum && a.maximum == b.maximum && (a.closed != 0) == (b.closed != 0)))
    return false;
  if (a.pattern_kind != b.pattern_kind) return false;
  if (a.pattern_kind != RT_PATTERN_NONE) {
    if (!m16_eq(a.pattern_transform, b.pattern_transform) ||
        !m16_eq(a.pattern_inverse, b.pattern_inverse))
      return false;
    if (a.pattern_kind != RT_PATTERN_TEST && !(c3_eq(a.pattern_a, b.pattern_a) && c3_eq(a.pattern_b, b.pattern_b)))
      return false;
  }
  return true;
}

int find_duplicate(const rt_shape_desc* s, size_t n, size_t* ia, size_t* ib) {
  std::vector<size_t> idx(n);
  for (size_t i = 0; i < n; ++i) idx[i] = i;
  // equal shapes have |translation-x difference| < EPSILON: sweep a sorted key
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return s[a].transform[3] < s[b].transform[3]; });
  for (size_t p = 0; p < n; ++p)
    for (size_t q = p + 1; q < n && s[idx[q]].transform[3] - s[idx[p]].transform[3] < rt::EPSILON; ++q)
      if (may_be_equal(s[idx[p]], s[idx[q]])) {
        *ia = std::min(idx[p], idx[q]);
        *ib = std::max(idx[p], idx[q]);
        return 1;
      }
  return 0;
}

}  // namespace

extern "C" {

int rt_scene_create(const rt_shape_desc* shapes, size_t n_shapes, const rt_light_desc* lights,
                    size_t n_lights, int device, rt_scene** out) {
  return guarded([&]() -> int {
  return rt_scene_create_groups(shapes, n_shapes, nullptr, nullptr, 0, lights, n_lights, device, out);
  });
}

int rt_scene_create_groups(const rt_shape_desc* shapes, size_t n_shapes, const int32_t* shape_group,
                           const rt_group_desc* groups, size_t n_groups, const rt_light_desc* lights,
                           size_t n_lights, int device, rt_scene** out) {
  return guarded([&]() -> int {
  if (!out || (n_shapes && !shapes) || (n_lights && !lights) || (n_groups && (!groups || !shape_group)))
    return fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  *out = nullptr;
  if (n_shapes > (size_t)(1u << 29)) return fail(RT_ERR_INVALID_ARGUMENT, "too many shapes");
  if (n_groups > (size_t)(1u << 24)) return fail(RT_ERR_INVALID_ARGUMENT, "too many groups");
  for (size_t g = 0; g < n_groups; ++g)
    if (groups[g].parent < -1 || groups[g].parent >= (int32_t)g)
      return fail(RT_ERR_INVALID_ARGUMENT, "group " + std::to_string(g) + ": its parent must be -1 or an earlier group");
  // a shape's gate: 1 + its innermost group (0: none)
  // (range-checked before the + 1: a caller's INT32_MAX must not overflow)
  for (size_t i = 0; shape_group && n_groups && i < n_shapes; ++i)
    if (shape_group[i] < -1 || (int64_t)shape_group[i] >= (int64_t)n_groups)
      return fail(RT_ERR_INVALID_ARGUMENT, "shape " + std::to_string(i) + ": bad group index");
  auto gate_of = [&](size_t i) -> int32_t { return shape_group && n_groups ? shape_group[i] + 1 : 0; };
  for (size_t i = 0; i < n_shapes; ++i) {
    if (shapes[i].kind < RT_SHAPE_SPHERE || shapes[i].kind > RT_SHAPE_CONE)
      return fail(RT_ERR_UNSUPPORTED_SHAPE, "shape " + std::to_string(i) +
                                                ": supported kinds are Sphere, Plane, Cube, Cylinder, Cone");
    if (shapes[i].pattern_kind < RT_PATTERN_NONE || shapes[i].pattern_kind > RT_PATTERN_CHECKERS)
      return fail(RT_ERR_INVALID_ARGUMENT, "shape " + std::to_string(i) + ": bad pattern kind");
  }
  size_t da, db;
  if (find_duplicate(shapes, n_shapes, &da, &db))
    return fail(RT_ERR_DUPLICATE_SHAPES, "shapes " + std::to_string(da) + " and " + std::to_string(db) +
                                             " may be structurally equal (containers walk, intersection.rs:63-90)");

  int ndev = rt_device_count();
  if (ndev <= 0) return fail(RT_ERR_NO_DEVICE, "no HIP device available (no CPU fallback)");
  if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID_ARGUMENT, "bad device ordinal");

  // ---- flatten (reference object order preserved through `meta`)
  std::vector<SphereDiag> diag;
  std::vector<SphereGen> gen;
  std::vector<PlaneRec> planes;
  std::vector<QuadRec> quads;
  std::vector<ShadeRec> shade(n_shapes);
  for (size_t i = 0; i < n_shapes; ++i) {
    const rt_shape_desc& d = shapes[i];
    const int64_t meta = ((int64_t)i << 1) | (d.casts_shadow ? 1 : 0);
    const int32_t gate = gate_of(i);  // shapes inside groups: general records with their group gate
    if (d.kind == RT_SHAPE_SPHERE) {
      if (is_diag_inverse(d.inverse) && gate == 0) {
        SphereDiag r{};
        r.s[0] = d.inverse[0]; r.s[1] = d.inverse[5]; r.s[2] = d.inverse[10];
        r.t[0] = d.inverse[3]; r.t[1] = d.inverse[7]; r.t[2] = d.inverse[11];
        r.meta = meta;
        diag.push_back(r);
      } else {
        SphereGen r{};
        for (int e = 0; e < 12; ++e) r.m[e] = d.inverse[e];
        r.meta = meta;
        r.gate = gate;
        gen.push_back(r);
      }
    } else if (d.kind == RT_SHAPE_PLANE) {
      PlaneRec r{};
      for (int e = 0; e < 4; ++e) r.m[e] = d.inverse[4 + e];
      r.meta = meta;
      r.gate = gate;
      planes.push_back(r);
    } else {
      QuadRec r{};
      for (int e = 0; e < 12; ++e) r.m[e] = d.inverse[e];
      r.minimum = d.minimum;
      r.maximum = d.maximum;
      r.kind = d.kind;
      r.closed = d.closed ? 1 : 0;
      r.meta = (int32_t)meta;
      r.gate = gate;
      quads.push_back(r);
    }
    ShadeRec& s = shade[i];
    std::memset(&s, 0, sizeof s);
    for (int e = 0; e < 12; ++e) s.inv[e] = d.inverse[e];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) s.invT[r * 3 + c] = d.inverse[c * 4 + r];  // transpose (matrix.rs:79-89)
    for (int c = 0; c < 3; ++c) s.color[c] = d.color[c];
    s.ambient = d.ambient; s.diffuse = d.diffuse; s.specular = d.specular; s.shininess = d.shininess;
    s.reflective = d.reflective; s.transparency = d.transparency; s.refractive_index = d.refractive_index;
    s.pattern_kind = d.pattern_kind;
    for (int c = 0; c < 3; ++c) { s.pat_a[c] = d.pattern_a[c]; s.pat_b[c] = d.pattern_b[c]; }
    for (int e = 0; e < 12; ++e) s.pat_inv[e] = d.pattern_inverse[e];
    s.kind = d.kind;
    s.shadow = d.casts_shadow ? 1 : 0;
    s.minimum = d.minimum;
    s.maximum = d.maximum;
  }
  // exact-culling hierarchy over the diagonal spheres (reorders `diag`; keys
  // come from `meta`, so the order changes no result)
  int bvh_depth = 0;
  const int leaf = g_bvh_leaf > 0 ? g_bvh_leaf : 2;
  std::vector<BvhNode> bvh = build_sphere_bvh(diag, leaf, &bvh_depth, g_bvh_ct / 100.0);
  if (g_bvh_leaf == 0 && !bvh.empty()) {
    // a scene whose pair image (stack, nodes, sphere records) does not fit in
    // LDS is traversed from global memory, where single-sphere leaves win
    const size_t image = (size_t)(bvh_depth + 1) * kFusedBlockThreads * 4 + bvh.size() * sizeof(BvhNode) +
                         diag.size() * sizeof(SphereDiag);
    if (image > kFusedLdsLimit) bvh = build_sphere_bvh(diag, 1, &bvh_depth, g_bvh_ct / 100.0);
  }
  const std::vector<BvhPair> bvh_pair = pair_layout(bvh);
  int wide_stack = 0;
  const std::vector<BvhWide> bvh_wide = wide_layout(bvh, diag, &wide_stack);
  const std::vector<BvhWide16> bvh_wide16 = wide16_layout(bvh_wide);
  // ... and over the other bounded records (general spheres, cubes, cylinders
  // with finite caps); the rest stays exhaustive on the fast path too
  std::vector<OtherRec> orec;
  std::vector<SphereGen> fx_gen;
  std::vector<QuadRec> fx_quads;
  double blo[3], bhi[3];
  // (shapes inside groups too: their group gate goes with them, tested before the
  // shape at the leaf, as the reference tests a group's box before its children)
  for (const SphereGen& g : gen) {
    OtherRec r{};
    for (int e = 0; e < 12; ++e) r.m[e] = g.m[e];
    r.kind = 0;
    r.meta = (int32_t)g.meta;
    r.gate = g.gate;
    if (other_box(r, blo, bhi)) orec.push_back(r);
    else fx_gen.push_back(g);
  }
  std::vector<QuadRec> line_rec;  // open tubes and cones with finite bounds: the line hierarchy
  for (const QuadRec& q : quads) {
    if (other_box(q, blo, bhi)) orec.push_back(q);
    else if (q.gate == 0 && line_box(q, blo, bhi)) line_rec.push_back(q);  // (grouped tubes and cones: exhaustive)
    else fx_quads.push_back(q);
  }
  std::vector<GroupRec> grec(n_groups);
  for (size_t g = 0; g < n_groups; ++g) {
    for (int c = 0; c < 3; ++c) { grec[g].lo[c] = groups[g].min[c]; grec[g].hi[c] = groups[g].max[c]; }
    grec[g].parent = groups[g].parent + 1;
  }
  // A handful of records is cheaper in the exhaustive loops (wave-uniform, scalar loads) than
  // behind a per-lane walk from global memory: the hierarchies start at kMinHierRecords
  // (640x480 frames: the groups scene's 7 grouped records 0.92 ms in the hierarchies, 0.69
  // exhaustive; solids 0.72 -> 0.60, zoo 0.37 -> 0.29; a divided group of 800: 5.1 against
  // 32.3), except in a scene without any other hierarchy, where one of
  // them is what opens the fused generations (the hexagon demo: 1.0 -> 0.53 ms)
  constexpr size_t kMinHierRecords = 16;
  int obvh_depth = 0;
  std::vector<BvhNode> obvh;
  if (orec.size() >= kMinHierRecords || (bvh.empty() && !orec.empty()))
    obvh = build_other_bvh(orec, leaf, &obvh_depth, g_bvh_ct / 100.0);
  if (obvh_depth > kBvhMaxDepth) obvh.clear();  // deeper than other_trace's stack: exhaustive
  int lbvh_depth = 0;
  std::vector<ConeCluster> lclus;
  std::vector<int32_t> lcone;
  std::vector<BvhNode> lbvh;
  if (line_rec.size() >= kMinHierRecords || (bvh.empty() && obvh.empty() && !line_rec.empty()))
    lbvh = build_line_bvh(line_rec, &lclus, &lcone, &lbvh_depth);
  if (lbvh.empty() || lbvh_depth > kBvhMaxDepth) {  // exhaustive, as before the line hierarchy
    for (const QuadRec& q : line_rec) fx_quads.push_back(q);
    line_rec.clear();
    lbvh.clear();
    lclus.clear();
    lcone.clear();
  }
  std::vector<int32_t> lrec_clus(line_rec.size(), -1);  // each cone's cluster (line_trace's pre-pass check)
  for (size_t c = 0; c < lclus.size(); ++c)
    for (int32_t j = lclus[c].first; j < lclus[c].first + lclus[c].count; ++j) lrec_clus[(size_t)lcone[(size_t)j]] = (int32_t)c;
  if (obvh.empty()) {  // (only when there are no records, or more than the leaf codes can index)
    for (const OtherRec& r : orec) {
      if (r.kind == 0) {
        SphereGen g{};
        for (int e = 0; e < 12; ++e) g.m[e] = r.m[e];
        g.meta = r.meta;
        g.gate = r.gate;
        fx_gen.push_back(g);
      } else {
        fx_quads.push_back(r);
      }
    }
    orec.clear();
  }
  std::vector<LightRec> lrec(n_lights);
  for (size_t i = 0; i < n_lights; ++i)
    for (int c = 0; c < 3; ++c) { lrec[i].pos[c] = lights[i].position[c]; lrec[i].intensity[c] = lights[i].intensity[c]; }
  // light buffers over the (reordered) diagonal spheres: the shadow rays' cell lists
  LightBuffer lb;
  const int lb_res = g_lb_res >= 0 ? g_lb_res : (diag.size() > 4096 ? 512 : 256);
  if (!diag.empty() && n_lights > 0 && n_lights <= (size_t)kLbMaxLights && lb_res > 0)
    lb = build_light_buffer(diag, lrec, lb_res);

  // ---- one blob, 64-B aligned sections
  auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_diag = 0;
  // one zeroed padding record after each trace section (look-ahead loads)
  const size_t o_gen = align(o_diag + (diag.size() + 1) * sizeof(SphereDiag));
  const size_t o_pl = align(o_gen + (gen.size() + 1) * sizeof(SphereGen));
  const size_t o_qd = align(o_pl + (planes.size() + 1) * sizeof(PlaneRec));
  const size_t o_bv = align(o_qd + (quads.size() + 1) * sizeof(QuadRec));
  const size_t o_bp = align(o_bv + (bvh.size() + 1) * sizeof(BvhNode));
  const size_t o_bw = align(o_bp + (bvh_pair.size() + 1) * sizeof(BvhPair));
  const size_t o_bh = align(o_bw + (bvh_wide.size() + 1) * sizeof(BvhWide));
  const size_t o_ob = align(o_bh + (bvh_wide16.size() + 1) * sizeof(BvhWide16));
  const size_t o_or = align(o_ob + (obvh.size() + 1) * sizeof(BvhNode));
  const size_t o_lb = align(o_or + (orec.size() + 1) * sizeof(OtherRec));
  const size_t o_lr = align(o_lb + (lbvh.size() + 1) * sizeof(BvhNode));
  const size_t o_cc = align(o_lr + (line_rec.size() + 1) * sizeof(QuadRec));
  const size_t o_lm = align(o_cc + (lclus.size() + 1) * sizeof(ConeCluster));
  const size_t o_lk = align(o_lm + (lcone.size() + 1) * sizeof(int32_t));
  const size_t o_fg = align(o_lk + (lrec_clus.size() + 1) * sizeof(int32_t));
  const size_t o_fq = align(o_fg + (fx_gen.size() + 1) * sizeof(SphereGen));
  const size_t o_sh = align(o_fq + (fx_quads.size() + 1) * sizeof(QuadRec));
  const size_t o_rt = align(o_sh + shade.size() * sizeof(ShadeRec));
  const size_t o_od = align(o_rt + (shade.size() + 1) * 2 * sizeof(double));
  const size_t o_li = align(o_od + (shade.size() + 1) * sizeof(int32_t));
  const size_t o_lc = align(o_li + lrec.size() * sizeof(LightRec));
  const size_t o_lv = align(o_lc + lb.cells.size() * sizeof(LbCell));
  const size_t o_ld = align(o_lv + (lb.ov.size() + 1) * sizeof(uint16_t));
  const size_t o_ll = align(o_ld + lb.delta.size() * sizeof(float));
  const size_t o_gr = align(o_ll + lb.limit.size() * sizeof(float));
  const size_t total = align(o_gr + grec.size() * sizeof(GroupRec)) + 256;
  std::vector<unsigned char> host(total, 0);
  if (!diag.empty()) std::memcpy(&host[o_diag], diag.data(), diag.size() * sizeof(SphereDiag));
  if (!gen.empty()) std::memcpy(&host[o_gen], gen.data(), gen.size() * sizeof(SphereGen));
  if (!planes.empty()) std::memcpy(&host[o_pl], planes.data(), planes.size() * sizeof(PlaneRec));
  if (!quads.empty()) std::memcpy(&host[o_qd], quads.data(), quads.size() * sizeof(QuadRec));
  if (!bvh.empty()) std::memcpy(&host[o_bv], bvh.data(), bvh.size() * sizeof(BvhNode));
  if (!bvh_pair.empty()) std::memcpy(&host[o_bp], bvh_pair.data(), bvh_pair.size() * sizeof(BvhPair));
  if (!bvh_wide.empty()) std::memcpy(&host[o_bw], bvh_wide.data(), bvh_wide.size() * sizeof(BvhWide));
  if (!bvh_wide16.empty()) std::memcpy(&host[o_bh], bvh_wide16.data(), bvh_wide16.size() * sizeof(BvhWide16));
  if (!obvh.empty()) std::memcpy(&host[o_ob], obvh.data(), obvh.size() * sizeof(BvhNode));
  if (!orec.empty()) std::memcpy(&host[o_or], orec.data(), orec.size() * sizeof(OtherRec));
  if (!lbvh.empty()) std::memcpy(&host[o_lb], lbvh.data(), lbvh.size() * sizeof(BvhNode));
  if (!lclus.empty()) std::memcpy(&host[o_cc], lclus.data(), lclus.size() * sizeof(ConeCluster));
  if (!lcone.empty()) std::memcpy(&host[o_lm], lcone.data(), lcone.size() * sizeof(int32_t));
  if (!lrec_clus.empty()) std::memcpy(&host[o_lk], lrec_clus.data(), lrec_clus.size() * sizeof(int32_t));
  if (!line_rec.empty()) std::memcpy(&host[o_lr], line_rec.data(), line_rec.size() * sizeof(QuadRec));
  if (!fx_gen.empty()) std::memcpy(&host[o_fg], fx_gen.data(), fx_gen.size() * sizeof(SphereGen));
  if (!fx_quads.empty()) std::memcpy(&host[o_fq], fx_quads.data(), fx_quads.size() * sizeof(QuadRec));
  if (!shade.empty()) std::memcpy(&host[o_sh], shade.data(), shade.size() * sizeof(ShadeRec));
  for (size_t i = 0; i < shade.size(); ++i) {
    const double rt2[2] = {shade[i].reflective, shade[i].transparency};
    std::memcpy(&host[o_rt + i * 2 * sizeof(double)], rt2, sizeof rt2);
  }
  {  // each object's SphereDiag record after the hierarchy's reordering (meta = object << 1 | shadow),
     // flagged kOwnOutside when its own shadow test may be left out for a hit from outside
     // (rt_trace.hpp, shadow_trace): the over point then lies EPSILON off the surface in world
     // space, at least EPSILON / r_max in object space, far above every rounding in the sphere
     // test when the semi-axes are at most 1e3 and the extent at most 1e6 (the over point's
     // EPSILON step resolved to 1e-10)
    std::vector<int32_t> obj_diag(shade.size() + 1, -1);
    for (size_t k = 0; k < diag.size(); ++k) {
      const SphereDiag& r = diag[k];
      bool own = true;
      for (int a = 0; a < 3; ++a) {
        const double sa = std::fabs(r.s[a]), ra = 1.0 / sa, ca = std::fabs(r.t[a] / r.s[a]);
        own = own && std::isfinite(ra) && std::isfinite(ca) && ra <= 1e3 && ca + ra <= 1e6;
      }
      obj_diag[(size_t)(r.meta >> 1)] = (int32_t)k | (own ? kOwnOutside : 0);
    }
    std::memcpy(&host[o_od], obj_diag.data(), obj_diag.size() * sizeof(int32_t));
  }
  if (!lrec.empty()) std::memcpy(&host[o_li], lrec.data(), lrec.size() * sizeof(LightRec));
  if (!grec.empty()) std::memcpy(&host[o_gr], grec.data(), grec.size() * sizeof(GroupRec));
  if (!lb.cells.empty()) {
    std::memcpy(&host[o_lc], lb.cells.data(), lb.cells.size() * sizeof(LbCell));
    if (!lb.ov.empty()) std::memcpy(&host[o_lv], lb.ov.data(), lb.ov.size() * sizeof(uint16_t));
    std::memcpy(&host[o_ld], lb.delta.data(), lb.delta.size() * sizeof(float));
    std::memcpy(&host[o_ll], lb.limit.data(), lb.limit.size() * sizeof(float));
  }

  rt_scene* s = new rt_scene();
  s->device = device;
  // children per ray at most (WfSizing::branch): the exact bound of the arenas
  int branch = 0;
  for (size_t i = 0; i < n_shapes; ++i)
    branch = std::max(branch, (shapes[i].reflective != 0.0 ? 1 : 0) + (shapes[i].transparency != 0.0 ? 1 : 0));
  s->sizing.branch = branch;
  s->band_sizing.branch = branch;
  {
    std::lock_guard<std::mutex> tlk(g_tune_mu);
    s->tune = g_tune_defaults;
  }
  auto cleanup = [&](int rc) {
    rt_scene_destroy(s);
    return rc;
  };
  int rc;
  DeviceGuard restore;  // the caller's device, whatever happens below
  if ((rc = [&]() -> int {
         RT_HIP(hipSetDevice(device));
         RT_HIP(hipMalloc(&s->d_blob, total));
         RT_HIP(hipMemcpy(s->d_blob, host.data(), total, hipMemcpyHostToDevice));
         RT_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
         return RT_OK;
       }()) != RT_OK)
    return cleanup(rc);
  unsigned char* b = (unsigned char*)s->d_blob;
  s->dev.sph_diag = (const SphereDiag*)(b + o_diag);
  s->dev.sph_gen = (const SphereGen*)(b + o_gen);
  s->dev.planes = (const PlaneRec*)(b + o_pl);
  s->dev.quads = (const QuadRec*)(b + o_qd);
  s->dev.bvh = bvh.empty() ? nullptr : (const BvhNode*)(b + o_bv);
  s->dev.bvh_pair = bvh_pair.empty() ? nullptr : (const BvhPair*)(b + o_bp);
  s->dev.bvhw = bvh_wide.empty() ? nullptr : (const BvhWide*)(b + o_bw);
  s->dev.bvhw16 = bvh_wide16.empty() ? nullptr : (const BvhWide16*)(b + o_bh);
  s->dev.n_bvhw = (int32_t)bvh_wide.size();
  s->dev.bvhw_stack = wide_stack;
  s->dev.n_bvh = (int32_t)bvh.size();
  s->dev.bvh_depth = bvh_depth;
  s->dev.obvh = obvh.empty() ? nullptr : (const BvhNode*)(b + o_ob);
  s->dev.orec = (const OtherRec*)(b + o_or);
  s->dev.lbvh = lbvh.empty() ? nullptr : (const BvhNode*)(b + o_lb);
  s->dev.lclus = (const ConeCluster*)(b + o_cc);
  s->dev.lcone = (const int32_t*)(b + o_lm);
  s->dev.lrec_clus = (const int32_t*)(b + o_lk);
  s->dev.n_lclus = (int32_t)lclus.size();
  s->dev.lrec = (const QuadRec*)(b + o_lr);
  s->dev.n_lbvh = (int32_t)lbvh.size();
  s->dev.n_lrec = (int32_t)line_rec.size();
  s->dev.n_obvh = (int32_t)obvh.size();
  s->dev.obvh_depth = obvh_depth;
  s->dev.n_orec = (int32_t)orec.size();
  s->dev.fx_gen = (const SphereGen*)(b + o_fg);
  s->dev.fx_quads = (const QuadRec*)(b + o_fq);
  s->dev.n_fx_gen = (int32_t)fx_gen.size();
  s->dev.n_fx_quads = (int32_t)fx_quads.size();
  s->dev.lb_cells = lb.cells.empty() ? nullptr : (const LbCell*)(b + o_lc);
  s->dev.lb_ov = (const uint16_t*)(b + o_lv);
  s->dev.lb_delta = (const float*)(b + o_ld);
  s->dev.lb_limit = (const float*)(b + o_ll);
  s->dev.lb_res = lb.res;
  s->dev.lb_n_items = (int32_t)std::min<size_t>(lb.n_items, 0x7FFFFFFF);
  s->dev.shade = (const ShadeRec*)(b + o_sh);
  s->dev.refl_transp = (const double*)(b + o_rt);
  s->dev.obj_diag = (const int32_t*)(b + o_od);
  s->dev.lights = (const LightRec*)(b + o_li);
  s->dev.groups = (const GroupRec*)(b + o_gr);
  s->dev.n_groups = (int32_t)n_groups;
  s->dev.n_diag = (int32_t)diag.size();
  s->dev.n_gen = (int32_t)gen.size();
  s->dev.n_planes = (int32_t)planes.size();
  s->dev.n_quads = (int32_t)quads.size();
  s->dev.n_objects = (int32_t)n_shapes;
  s->dev.n_lights = (int32_t)n_lights;
  s->n_objects = (int)n_shapes;
  s->n_lights = (int)n_lights;
  *out = s;
  return RT_OK;
  });
}

void rt_scene_destroy(rt_scene* s) {
  if (!s) return;
  DeviceGuard restore(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  s->multi.release();
  (void)hipSetDevice(s->device);
  if (s->d_blob) (void)hipFree(s->d_blob);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;  // the host contexts and workspaces release their memory (on the scene's device)
}

}  // extern "C"
