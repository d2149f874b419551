// Host check of rt_bvh.cpp's four-wide layout (tests/test_bvh_host.py):
// random sphere fields (C3/C5-like), every leaf size the builder takes.
// Checks that every record is reached exactly once, that every slot's box
// holds the records below it (each record's padded box, so the culling stays
// exact), that child codes are 16-bit, and that a near-first traversal of
// random rays never keeps more entries pending than the reported stack bound;
// that the binary16 copy (wide16_layout) holds the same codes and boxes that
// hold the binary32 ones; and the binary16 outward rounding itself.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "rt_bvh.hpp"

using namespace rtamd;

static int fail(const char* what, int a, int b) {
  std::printf("FAIL %s %d %d\n", what, a, b);
  return 1;
}

// f16_bits_down / f16_bits_up: the nearest binary16 at or below / above x
// (normal or zero, an infinity past the range), checked against the spacing
static int check_f16() {
  std::mt19937_64 g(99);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (int i = 0; i < 200000; ++i) {
    const double x = u(g) * std::ldexp(1.0, (int)(g() % 44) - 24);
    const float d = wide_f16(f16_bits_down(x)), up = wide_f16(f16_bits_up(x));
    if (!((double)d <= x && (double)up >= x)) return fail("f16 side", i, 0);
    const double ax = std::fabs(x);
    if (ax >= 0x1p-14 && ax <= 65504.0) {
      int e;
      std::frexp(ax, &e);
      const double sp = std::ldexp(1.0, e - 11);  // one binary16 step at |x|
      if (x - d >= sp || up - x >= sp) return fail("f16 step", i, 0);
    }
    if (ax > 65504.0 && !(x > 0 ? std::isinf(up) && d == 65504.0f : std::isinf(d) && up == -65504.0f))
      return fail("f16 range", i, 0);
    if (ax < 0x1p-14 && !(x >= 0 ? d == 0.0f && up <= 0x1p-14f : d == -0x1p-14f && up == 0.0f)) return fail("f16 tiny", i, 0);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (check_f16()) return 1;
  const int n = std::atoi(argv[1]), leaf = std::atoi(argv[2]);
  const double span = argc > 3 ? std::atof(argv[3]) : 50.0;
  std::mt19937_64 g(1234 + n * 7 + leaf);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<SphereDiag> sp(n);
  for (int i = 0; i < n; ++i) {
    const double r = 0.15 + 0.35 * u(g), c[3] = {span * (u(g) - 0.5), r + 0.6 * span * u(g), span * (u(g) - 0.2)};
    for (int a = 0; a < 3; ++a) {
      sp[i].s[a] = 1.0 / r;
      sp[i].t[a] = -c[a] / r;
    }
    sp[i].meta = i;
  }
  int depth = 0, stack = 0;
  const std::vector<BvhNode> b = build_sphere_bvh(sp, leaf, &depth, 1.0);
  const std::vector<BvhWide> w = wide_layout(b, sp, &stack);
  if (w.empty()) return fail("empty", n, leaf);
  const std::vector<BvhWide16> w16 = wide16_layout(w);
  if (w16.size() != w.size()) return fail("size16", (int)w16.size(), (int)w.size());
  if (w.size() >= 0x8000) return fail("nodes", (int)w.size(), 0);
  std::vector<int> seen(n, 0), refs(w.size(), 0);
  // containment and coverage: walk from the root
  std::vector<int> todo{0};
  while (!todo.empty()) {
    const int e = todo.back();
    todo.pop_back();
    for (int j = 0; j < 4; ++j) {
      const unsigned c = (unsigned)w[e].child[j];
      if (c == kWideEmpty) continue;
      if (c > 0xFFFFu) return fail("code", e, j);
      float lo[3], hi[3];
      for (int a = 0; a < 3; ++a) {
        lo[a] = w[e].lo[a][j];
        hi[a] = w[e].hi[a][j];
        // the global-memory copy's binary16 box holds the binary32 one
        if (!(wide_f16(w16[e].lo[a][j]) <= lo[a] && wide_f16(w16[e].hi[a][j]) >= hi[a])) return fail("box16", e, j);
      }
      if (w16[e].child[j] != w[e].child[j]) return fail("code16", e, j);
      std::vector<int> below;
      if (c & kWideLeaf) {
        below.push_back((int)(c & 0x7FFFu));
        ++seen[c & 0x7FFFu];
      } else {
        if ((size_t)c >= w.size()) return fail("index", e, (int)c);
        ++refs[c];
        todo.push_back((int)c);
        std::vector<int> sub{(int)c};  // records below node c
        while (!sub.empty()) {
          const int f = sub.back();
          sub.pop_back();
          for (int k = 0; k < 4; ++k) {
            const unsigned d = (unsigned)w[f].child[k];
            if (d == kWideEmpty) continue;
            if (d & kWideLeaf) below.push_back((int)(d & 0x7FFFu));
            else sub.push_back((int)d);
          }
        }
      }
      for (int k : below)
        for (int a = 0; a < 3; ++a) {
          const double cen = -sp[k].t[a] / sp[k].s[a], r = 1.0 / sp[k].s[a];
          if (!((double)lo[a] < cen - r && (double)hi[a] > cen + r)) return fail("box", e, k);
        }
    }
  }
  for (int k = 0; k < n; ++k)
    if (seen[k] != 1) return fail("record", k, seen[k]);
  for (size_t i = 1; i < w.size(); ++i)
    if (refs[i] != 1) return fail("node refs", (int)i, refs[i]);
  // pending entries of a near-first walk (every box the ray's line meets is
  // visited: the most a culling walk could push)
  int most = 0;
  for (int q = 0; q < 2000; ++q) {
    double o[3] = {span * (u(g) - 0.5), span * 0.3 * u(g), -span}, d[3];
    for (int a = 0; a < 3; ++a) d[a] = u(g) - 0.5;
    d[2] = std::fabs(d[2]) + 0.2;
    std::vector<int> st;
    int e = 0;
    for (;;) {
      if (e >= 0) {
        std::vector<std::pair<double, int>> hit;
        for (int j = 0; j < 4; ++j) {
          const unsigned c = (unsigned)w[e].child[j];
          if (c == kWideEmpty) continue;
          double t0 = 0.0, t1 = INFINITY;
          for (int a = 0; a < 3; ++a) {
            const double inv = 1.0 / d[a];
            double ta = (w[e].lo[a][j] - o[a]) * inv, tb = (w[e].hi[a][j] - o[a]) * inv;
            if (ta > tb) std::swap(ta, tb);
            t0 = std::max(t0, ta);
            t1 = std::min(t1, tb);
          }
          if (t0 <= t1) hit.push_back({t0, (c & kWideLeaf) ? -1 : (int)c});
        }
        std::sort(hit.begin(), hit.end());
        for (size_t k = hit.size(); k-- > 1;) st.push_back(hit[k].second);
        most = std::max(most, (int)st.size());
        if (!hit.empty()) { e = hit[0].second; continue; }
      }
      if (st.empty()) break;
      e = st.back();
      st.pop_back();
    }
  }
  if (most > stack) return fail("stack", most, stack);
  std::printf("OK n=%d leaf=%d nodes=%zu stack=%d most=%d depth=%d\n", n, leaf, w.size(), stack, most, depth);
  return 0;
}
