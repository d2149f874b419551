// Host check of rt_bvh.cpp's light buffer (tests/test_bvh_host.py): every
// cell's list is ordered by (binary32 box distance, record index), the inline
// entries and the overflow lists agree with the counts, and every
// shadow-casting record is listed in the cell of the direction from each light
// to its centre (the cell a shadow ray towards that light through the centre
// reads).
#include <algorithm>
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

int main(int argc, char** argv) {
  const int n = std::atoi(argv[1]), R = std::atoi(argv[2]);
  std::mt19937_64 g(77 + n + R);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  std::vector<SphereDiag> sp(n);
  for (int i = 0; i < n; ++i) {
    const double r = 0.15 + 0.35 * u(g), c[3] = {-25 + 50 * u(g), r + 30 * u(g), -10 + 40 * u(g)};
    for (int a = 0; a < 3; ++a) { sp[i].s[a] = 1.0 / r; sp[i].t[a] = -c[a] / r; }
    sp[i].meta = ((int64_t)i << 1) | (i % 5 ? 1 : 0);
  }
  std::vector<LightRec> L(2);
  const double p[2][3] = {{-10, 25, -20}, {15, 20, -15}};
  for (int l = 0; l < 2; ++l)
    for (int a = 0; a < 3; ++a) { L[l].pos[a] = p[l][a]; L[l].intensity[a] = 1.0; }
  const LightBuffer lb = build_light_buffer(sp, L, R);
  const size_t per = (size_t)6 * R * R;
  if (lb.cells.size() != 2 * per) return fail("cells", (long)lb.cells.size(), (long)per);
  size_t items = 0;
  auto entry = [&](const LbCell& c, size_t k) -> unsigned {
    const unsigned in[5] = {c.w0 >> 16, c.w1 & 0xFFFFu, c.w1 >> 16, c.w2 & 0xFFFFu, c.w2 >> 16};
    return k < 5 ? in[k] : lb.ov[c.ov + k - 5];
  };
  for (size_t l = 0; l < 2; ++l)
    for (size_t c = 0; c < per; ++c) {
      const LbCell& cell = lb.cells[l * per + c];
      const size_t m = cell.w0 & 0xFFFFu;
      items += m;
      if (m > 5 && cell.ov + (m - 5) > lb.ov.size()) return fail("ov", (long)c, (long)m);
      for (size_t k = 1; k < m; ++k) {
        const unsigned a = entry(cell, k - 1), b = entry(cell, k);
        const float da = lb.delta[l * n + a], db = lb.delta[l * n + b];
        if (!(da < db || (da == db && a < b))) return fail("order", (long)c, (long)k);
      }
    }
  if (items != lb.n_items) return fail("items", (long)items, (long)lb.n_items);
  // each caster in the cell of the direction light -> centre
  for (int i = 0; i < n; ++i) {
    if (!(sp[i].meta & 1)) continue;
    for (size_t l = 0; l < 2; ++l) {
      double w[3];
      for (int a = 0; a < 3; ++a) w[a] = -sp[i].t[a] / sp[i].s[a] - L[l].pos[a];
      int ax = 0;
      for (int a = 1; a < 3; ++a)
        if (std::fabs(w[a]) > std::fabs(w[ax])) ax = a;
      const int f = 2 * ax + (w[ax] < 0 ? 1 : 0), b = (ax + 1) % 3, cc = (ax + 2) % 3;
      const double uu = w[b] / std::fabs(w[ax]), vv = w[cc] / std::fabs(w[ax]);
      const int iu = std::min((int)((uu + 1.0) * 0.5 * R), R - 1), iv = std::min((int)((vv + 1.0) * 0.5 * R), R - 1);
      const LbCell& cell = lb.cells[l * per + ((size_t)f * R + iv) * R + iu];
      bool found = false;
      for (size_t k = 0; k < (cell.w0 & 0xFFFFu) && !found; ++k) found = entry(cell, k) == (unsigned)i;
      if (!found) return fail("listed", i, (long)l);
    }
  }
  std::printf("OK n=%d R=%d items=%zu ov=%zu\n", n, R, lb.n_items, lb.ov.size());
  return 0;
}
