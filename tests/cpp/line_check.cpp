// Host check of rt_bvh.cpp's line hierarchy (tests/test_bvh_host.py): random
// cones (upright ones of one scale, ones turned about their axis, and ones
// under random inverses) and open tubes. Checks that every record sits in
// exactly one leaf, that the clusters hold every cone once and only cones,
// and that the cluster tests are sound: for random directions and directions
// along each cone's generators (the reference's a ~ 0 branch,
// cone.rs:102-110), whenever a cone's a as the reference computes it is below
// EPSILON, its cluster's test is open (the device's cone_cluster_open,
// rt_trace.hpp, restated here).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "rt_bvh.hpp"

using namespace rtamd;

static int fail(const char* what, long a, long b) {
  std::printf("FAIL %s %ld %ld\n", what, a, b);
  return 1;
}

static bool gate_open(const ConeCluster& g, const double d[3]) {  // rt_trace.hpp cone_cluster_open
  const double dm = std::fmax(std::fmax(std::fabs(d[0]), std::fabs(d[1])), std::fabs(d[2])), dm2 = dm * dm;
  const double v = g.q[0] * d[0] * d[0] + g.q[1] * d[1] * d[1] + g.q[2] * d[2] * d[2] +
                   2.0 * (g.q[3] * d[0] * d[1] + g.q[4] * d[0] * d[2] + g.q[5] * d[1] * d[2]);
  const double av = std::fabs(v), rr = g.r * dm2;
  return !(av - rr - 0x1p-40 * (av + rr) >= kEpsilon);
}
static double cone_a(const QuadRec& q, const double d[3]) {  // quad_test's object direction, then a
  const double x = q.m[0] * d[0] + q.m[1] * d[1] + q.m[2] * d[2];
  const double y = q.m[4] * d[0] + q.m[5] * d[1] + q.m[6] * d[2];
  const double z = q.m[8] * d[0] + q.m[9] * d[1] + q.m[10] * d[2];
  return x * x - y * y + z * z;
}
// d = A^-1 v for the 3x3 part A of the inverse (a world direction whose object direction is v)
static void world_dir(const QuadRec& q, const double v[3], double d[3]) {
  const double* m = q.m;
  const double a[3][3] = {{m[0], m[1], m[2]}, {m[4], m[5], m[6]}, {m[8], m[9], m[10]}};
  const double c[3][3] = {{a[1][1] * a[2][2] - a[1][2] * a[2][1], a[0][2] * a[2][1] - a[0][1] * a[2][2],
                           a[0][1] * a[1][2] - a[0][2] * a[1][1]},
                          {a[1][2] * a[2][0] - a[1][0] * a[2][2], a[0][0] * a[2][2] - a[0][2] * a[2][0],
                           a[0][2] * a[1][0] - a[0][0] * a[1][2]},
                          {a[1][0] * a[2][1] - a[1][1] * a[2][0], a[0][1] * a[2][0] - a[0][0] * a[2][1],
                           a[0][0] * a[1][1] - a[0][1] * a[1][0]}};
  const double det = a[0][0] * c[0][0] + a[0][1] * c[1][0] + a[0][2] * c[2][0];
  for (int i = 0; i < 3; ++i) d[i] = (c[i][0] * v[0] + c[i][1] * v[1] + c[i][2] * v[2]) / det;
}

int main(int argc, char** argv) {
  const int n = std::atoi(argv[1]);
  const double upright = argc > 2 ? std::atof(argv[2]) : 0.5;
  std::mt19937_64 g(4321 + n);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  std::vector<QuadRec> recs(n);
  for (int i = 0; i < n; ++i) {
    QuadRec& q = recs[i];
    q = QuadRec{};
    const bool tube = i % 5 == 4;
    q.kind = tube ? 3 : 4;
    q.closed = tube ? 0 : (i % 2);
    q.minimum = -1.0 + 0.8 * (u(g) + 1.0) / 2.0;
    q.maximum = q.minimum + 0.3 + (u(g) + 1.0) / 2.0;
    q.meta = i << 1;
    const double t[3] = {8.0 * u(g), 3.0 + 2.0 * u(g), 8.0 * u(g)};
    const double pick = (u(g) + 1.0) / 2.0;
    if (!tube && pick < upright) {  // translation . scaling(0.4), turned about y by one of 4 angles: one Q
      const double k = 2.5, th = 1.5707963267948966 * (i % 4), cs = std::cos(th), sn = std::sin(th);
      const double m[12] = {k * cs, 0, -k * sn, 0, 0, k, 0, 0, k * sn, 0, k * cs, 0};
      for (int e = 0; e < 12; ++e) q.m[e] = m[e];
      for (int r = 0; r < 3; ++r) q.m[4 * r + 3] = -(q.m[4 * r] * t[0] + q.m[4 * r + 1] * t[1] + q.m[4 * r + 2] * t[2]);
    } else {
      for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) q.m[4 * r + c] = (r == c ? 2.0 : 0.0) + 0.8 * u(g);
        q.m[4 * r + 3] = -(q.m[4 * r] * t[0] + q.m[4 * r + 1] * t[1] + q.m[4 * r + 2] * t[2]);
      }
    }
  }
  std::vector<QuadRec> kept = recs;
  std::vector<ConeCluster> clus;
  std::vector<int32_t> members;
  int depth = 0;
  const std::vector<BvhNode> nodes = build_line_bvh(kept, &clus, &members, &depth);
  if (nodes.empty()) return fail("empty", n, 0);
  // leaves
  std::vector<int> seen(kept.size(), 0);
  std::vector<int> todo{0};
  while (!todo.empty()) {
    const int e = todo.back();
    todo.pop_back();
    for (int c = 0; c < 2; ++c) {
      const int32_t code = nodes[e].child[c];
      if (code == kBvhEmpty) continue;
      if (code >= 0) {
        todo.push_back(code);
        continue;
      }
      const int v = -(code + 1), first = v >> 7, cnt = v & 127;
      for (int k = first; k < first + cnt; ++k) ++seen[k];
    }
  }
  for (size_t k = 0; k < kept.size(); ++k)
    if (seen[k] != 1) return fail("record", (long)k, seen[k]);
  // clusters: every cone once, nothing else
  std::vector<int> cluster_of(kept.size(), -1);
  for (size_t c = 0; c < clus.size(); ++c)
    for (int j = clus[c].first; j < clus[c].first + clus[c].count; ++j) {
      const int k = members[j];
      if (kept[k].kind != 4 || cluster_of[k] >= 0) return fail("member", (long)c, k);
      cluster_of[k] = (int)c;
    }
  for (size_t k = 0; k < kept.size(); ++k)
    if (kept[k].kind == 4 && cluster_of[k] < 0) return fail("cone without cluster", (long)k, 0);
  // soundness
  long degenerate = 0, opened = 0, checks = 0;
  auto check = [&](const double d[3]) -> int {
    for (size_t k = 0; k < kept.size(); ++k) {
      if (kept[k].kind != 4) continue;
      ++checks;
      if (!(std::fabs(cone_a(kept[k], d)) < kEpsilon)) continue;
      ++degenerate;
      if (!gate_open(clus[cluster_of[k]], d)) return fail("cluster closed on a degenerate cone", (long)k, cluster_of[k]);
    }
    for (const ConeCluster& gt : clus) opened += gate_open(gt, d);
    return 0;
  };
  for (int q = 0; q < 3000; ++q) {
    double d[3] = {u(g), u(g), u(g)};
    if (check(d)) return 1;
  }
  for (size_t k = 0; k < kept.size(); ++k) {  // along the generators, and around them
    if (kept[k].kind != 4) continue;
    for (int j = 0; j < 12; ++j) {
      const double th = 0.5236 * j, eps = j % 3 == 0 ? 0.0 : (j % 3 == 1 ? 2e-6 : -3e-6);
      const double v[3] = {std::cos(th), (j % 2 ? 1.0 : -1.0) * (1.0 + eps), std::sin(th)};
      double d[3];
      world_dir(kept[k], v, d);
      const double s = (u(g) + 1.5) * 3.0;  // any length
      for (double& x : d) x *= s;
      if (check(d)) return 1;
    }
  }
  if (degenerate == 0) return fail("no degenerate direction exercised", 0, 0);
  std::printf("OK n=%d nodes=%zu depth=%d clusters=%zu checks=%ld degenerate=%ld clusters_open=%ld\n", n, nodes.size(),
              depth, clus.size(), checks, degenerate, opened);
  return 0;
}
