// Dev study (not built into the library): SAH cost of rt_bvh.cpp's four-wide
// collapse (wide_layout: open the largest-area slot until four) against the
// cost-optimal collapse of the same binary tree (dynamic programming over
// "this subtree as at most k slots", k = 1..4), on the C3 / C5 sphere fields.
// Cost = sum over visited wide nodes of P(visit) * c_visit + sum over record
// slots of P(test) * c_test, P = area / area(root).
// Usage: wide_sah [c3|c5] [c_visit] [c_test] [leaf] [f16]
// (f16: the greedy cost over the binary16 copy's boxes, wide16_layout)
// Build: g++ -O2 -std=c++17 -pthread -I raytracer-challenge-rs_amd/csrc tools/archive/wide_sah.cpp
//        raytracer-challenge-rs_amd/csrc/rt_bvh.cpp -o /tmp/wide_sah
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <array>
#include <string>
#include <vector>

#include "rt_bvh.hpp"

using namespace rtamd;

struct SplitMix {
  uint64_t s;
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double u() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

// scenes.c3 / scenes.c5 sphere draws (rtamd/scenes.py _random_sphere)
static std::vector<SphereDiag> field(int n, uint64_t seed, const double lo[3], const double hi[3]) {
  SplitMix g{seed};
  std::vector<SphereDiag> sp(n);
  for (int i = 0; i < n; ++i) {
    const double r = 0.15 + 0.35 * g.u();
    const double c[3] = {lo[0] + (hi[0] - lo[0]) * g.u(), r + (hi[1] - lo[1]) * g.u(), lo[2] + (hi[2] - lo[2]) * g.u()};
    const double k = g.u();
    if (k < 0.5) { g.u(); g.u(); g.u(); }
    else if (k < 0.8) { g.u(); }
    for (int a = 0; a < 3; ++a) { sp[i].s[a] = 1.0 / r; sp[i].t[a] = -c[a] / r; }
    sp[i].meta = i;
  }
  return sp;
}

struct B3 {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void add(const B3& o) {
    for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], o.lo[a]); hi[a] = std::max(hi[a], o.hi[a]); }
  }
  double area() const {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};
static B3 rec_box(const SphereDiag& r) {
  B3 b;
  for (int a = 0; a < 3; ++a) {
    const double p0 = (-1.0 - r.t[a]) / r.s[a], p1 = (1.0 - r.t[a]) / r.s[a];
    b.lo[a] = std::min(p0, p1);
    b.hi[a] = std::max(p0, p1);
  }
  return b;
}

// an item of the binary tree: a node's child slot (a node, a record range)
struct Item {
  B3 box;
  int a = -1, b = -1;  // children items (-1: a record)
};

int main(int argc, char** argv) {
  const bool c5 = argc > 1 && std::string(argv[1]) == "c5";
  const double cv = argc > 2 ? std::atof(argv[2]) : 1.0, ct = argc > 3 ? std::atof(argv[3]) : 1.0;
  const int leaf = argc > 4 ? std::atoi(argv[4]) : (c5 ? 1 : 2);
  std::vector<SphereDiag> sp;
  if (!c5) {
    const double lo[3] = {-10, 0, -2}, hi[3] = {10, 3, 20};
    sp = field(1000, 0x5EED0003ull, lo, hi);
  } else {
    const double lo[3] = {-25, 0, -10}, hi[3] = {25, 30, 30};
    sp = field(9996, 0x5EED0005ull, lo, hi);
  }
  int depth = 0, stack = 0;
  const std::vector<BvhNode> b = build_sphere_bvh(sp, leaf, &depth, 0.7);
  const std::vector<BvhWide> w = wide_layout(b, sp, &stack);
  const std::vector<BvhWide16> w16 = wide16_layout(w);
  const bool f16 = argc > 5 && std::string(argv[5]) == "f16";
  // root area: union of the root node's two child boxes
  B3 root;
  for (int c = 0; c < 2; ++c) {
    B3 x;
    for (int a = 0; a < 3; ++a) { x.lo[a] = b[0].lo[c][a]; x.hi[a] = b[0].hi[c][a]; }
    if (b[0].child[c] != kBvhEmpty) root.add(x);
  }
  const double A0 = root.area();
  // greedy (library) cost
  double greedy = cv;  // the root is always visited
  double gv = cv, gt = 0.0;  // the visit and test parts
  int wn = 0;
  {
    std::vector<int> todo{0};
    while (!todo.empty()) {
      const int e = todo.back();
      todo.pop_back();
      ++wn;
      for (int j = 0; j < 4; ++j) {
        const unsigned c = w[e].child[j];
        if (c == kWideEmpty) continue;
        B3 x;
        for (int a = 0; a < 3; ++a) {
          x.lo[a] = f16 ? wide_f16(w16[e].lo[a][j]) : w[e].lo[a][j];
          x.hi[a] = f16 ? wide_f16(w16[e].hi[a][j]) : w[e].hi[a][j];
        }
        const double p = x.area() / A0;
        if (c & kWideLeaf) { greedy += p * ct; gt += p * ct; }
        else { greedy += p * cv; gv += p * cv; todo.push_back((int)c); }
      }
    }
  }
  // items of the binary tree (record ranges split in halves down to single records)
  std::vector<Item> it;
  auto rec_range = [&](auto&& self, int first, int cnt) -> int {
    Item x;
    if (cnt == 1) {
      x.box = rec_box(sp[first]);
      it.push_back(x);
      return (int)it.size() - 1;
    }
    const int h = cnt / 2;
    const int l = self(self, first, h), r = self(self, first + h, cnt - h);
    x.a = l; x.b = r;
    x.box = it[l].box; x.box.add(it[r].box);
    it.push_back(x);
    return (int)it.size() - 1;
  };
  auto node_item = [&](auto&& self, int n) -> int {
    int ch[2] = {-1, -1};
    for (int c = 0; c < 2; ++c) {
      const int32_t code = b[n].child[c];
      if (code == kBvhEmpty) continue;
      if (code >= 0) ch[c] = self(self, code);
      else {
        const int v = -(code + 1);
        ch[c] = rec_range(rec_range, v >> 7, v & 127);
      }
    }
    if (ch[1] < 0) return ch[0];
    Item x;
    x.a = ch[0]; x.b = ch[1];
    x.box = it[ch[0]].box; x.box.add(it[ch[1]].box);
    it.push_back(x);
    return (int)it.size() - 1;
  };
  const int top = node_item(node_item, 0);
  // DP: C[i][k] = least cost of item i's subtree as at most k slots (k = 1..4)
  const size_t n = it.size();
  std::vector<std::array<double, 5>> C(n);
  for (size_t i = 0; i < n; ++i) {  // children precede parents in `it`
    const Item& x = it[i];
    const double p = x.box.area() / A0;
    if (x.a < 0) {
      for (int k = 1; k <= 4; ++k) C[i][k] = p * ct;
      continue;
    }
    double dist = INFINITY;  // a wide node over this item: its four slots split between the children
    for (int j = 1; j <= 3; ++j) dist = std::min(dist, C[x.a][j] + C[x.b][4 - j]);
    C[i][1] = p * cv + dist;
    for (int k = 2; k <= 4; ++k) {
      double best = C[i][k - 1];
      for (int j = 1; j < k; ++j) best = std::min(best, C[x.a][j] + C[x.b][k - j]);
      C[i][k] = best;
    }
  }
  const Item& r = it[top];
  double opt = INFINITY;
  for (int j = 1; j <= 3; ++j) opt = std::min(opt, C[r.a][j] + C[r.b][4 - j]);
  opt += cv;
  std::printf("%s leaf=%d c_visit=%.2f c_test=%.2f%s: greedy wide nodes=%d cost=%.3f (visits %.3f, tests %.3f)  optimal cost=%.3f  (%.1f%%)\n",
              c5 ? "C5" : "C3", leaf, cv, ct, f16 ? " (binary16 boxes)" : "", wn, greedy, gv, gt, opt,
              100.0 * (opt / greedy - 1.0));
  return 0;
}
