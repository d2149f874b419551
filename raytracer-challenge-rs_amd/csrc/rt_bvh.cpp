// rt_bvh.cpp — host-side BVHs over the flattened world's bounded records.
//
// The reference accelerates only through `Group` (bounding-box early-out,
// group.rs:50-70) and `Group::divide` (split the children by the halves of
// the group's box, group.rs:108-188; AABB slab test bounding_box.rs:95-136).
// This builder plays that role for the flattened world, with two changes
// that matter on the GPU:
//   * binned-SAH splits over the record centroids (32 bins, all three axes),
//     and
//   * every box is padded outward, so the traversal never culls a record the
//     exhaustive loop would have hit: culling is exact by construction
//     (DESIGN.md "Exact culling").
#include "rt_bvh.hpp"

#include <algorithm>
#include <array>
#include <map>
#include <cmath>
#include <cstring>
#include <limits>
#include <thread>

namespace rtamd {
namespace {

struct Box {
  double lo[3] = {INFINITY, INFINITY, INFINITY};
  double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  void grow(const double* p) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  double area() const {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

// Padding of a record's box: 1e-6 of its size and position (far above the
// rounding of any root computed from the record; DESIGN.md "Exact culling").
void pad_axis(double lo, double hi, double* out_lo, double* out_hi) {
  const double pad = 1e-6 * ((hi - lo) + std::fabs(lo) + std::fabs(hi)) + 1e-9;
  *out_lo = lo - pad;
  *out_hi = hi + pad;
}

// World-space extent of the record's unit sphere: the stored inverse maps
// p -> s*p + t per axis, and |s*p + t| <= 1 means p in [(-1-t)/s, (1-t)/s].
Box sphere_box(const SphereDiag& r) {
  Box b;
  for (int a = 0; a < 3; ++a) {
    const double p0 = (-1.0 - r.t[a]) / r.s[a];
    const double p1 = (1.0 - r.t[a]) / r.s[a];
    pad_axis(std::min(p0, p1), std::max(p0, p1), &b.lo[a], &b.hi[a]);
  }
  return b;
}

// binary32 rounded outward (the node boxes only ever grow)
float f32_down(double x) {
  float f = (float)x;
  if ((double)f > x) f = std::nextafter(f, -INFINITY);
  return f;
}
float f32_up(double x) {
  float f = (float)x;
  if ((double)f < x) f = std::nextafter(f, INFINITY);
  return f;
}
// binary16 rounded outward, as bit patterns (BvhWide): the largest binary16
// value <= x (f16_bits_down) or the smallest >= x (f16_bits_up); past the
// largest finite value, the infinity on that side
static uint16_t f16_bits(double q) {  // q: a binary16 value (or an infinity)
  const uint16_t sign = std::signbit(q) ? 0x8000u : 0u;
  const double a = std::fabs(q);
  if (std::isinf(a)) return sign | 0x7C00u;
  if (a < 0x1p-14) return sign;  // zero (f16_floor makes no subnormals)
  int e;
  const double m = std::frexp(a, &e);  // a = m 2^e, m in [0.5, 1)
  return sign | (uint16_t)((e + 14) << 10) | (uint16_t)((m * 2.0 - 1.0) * 1024.0);
}
// (no subnormal results: a value below the smallest normal goes to 0 or to
// -2^-14, so no flush of subnormal inputs can move a plane inward)
static double f16_floor(double x) {
  if (std::isnan(x)) return -INFINITY;
  if (std::isinf(x)) return x;
  const double ax = std::fabs(x);
  if (ax < 0x1p-14) return x >= 0.0 ? 0.0 : -0x1p-14;
  int e;
  std::frexp(ax, &e);
  const double u = std::ldexp(1.0, e - 11);  // the spacing at |x|
  const double q = std::floor(x / u) * u;
  return q < -65504.0 ? -INFINITY : q > 65504.0 ? 65504.0 : q;
}

// Binned-SAH builder over item boxes; produces the node array and the leaf
// order of the items (`order[k]` = original index of the k-th leaf item).
struct Builder {
  std::vector<int> order;
  std::vector<Box> box;
  std::vector<double> cen;  // 3 per item
  std::vector<BvhNode> nodes;
  int leaf_size;
  double trav_cost;  // SAH cost of a node visit relative to one record test

  static constexpr int kBins = 32;

  // Returns the child code for items [b, e) at `depth`.
  int32_t build(int b, int e, int depth, Box* out_box) {
    Box bb, cb;
    for (int i = b; i < e; ++i) {
      bb.grow(box[i]);
      cb.grow(&cen[3 * i]);
    }
    *out_box = bb;
    const int n = e - b;
    if (n <= leaf_size) return leaf(b, n);
    int axis = 0;
    double ext = -1;
    for (int a = 0; a < 3; ++a)
      if (cb.hi[a] - cb.lo[a] > ext) { ext = cb.hi[a] - cb.lo[a]; axis = a; }
    int mid = -1;
    if (ext > 0 && depth < kBvhMaxDepth - 24) {
      // binned SAH over the three centroid axes: split cost C_t * A + sum(A_side * n_side)
      double best = INFINITY;
      int best_k = -1, best_axis = axis;
      for (int ax = 0; ax < 3; ++ax) {
        const double ex = cb.hi[ax] - cb.lo[ax];
        if (!(ex > 0)) continue;
        Box bin_box[kBins];
        int bin_n[kBins] = {0};
        for (int i = b; i < e; ++i) {
          const int k = bin_index(i, ax, cb.lo[ax], ex);
          ++bin_n[k];
          bin_box[k].grow(box[i]);
        }
        Box right[kBins];
        int nright[kBins + 1] = {0};
        for (int k = kBins - 1; k >= 1; --k) {
          right[k] = k + 1 < kBins ? right[k + 1] : Box{};
          if (bin_n[k]) right[k].grow(bin_box[k]);
          nright[k] = nright[k + 1] + bin_n[k];
        }
        Box l;
        int nl = 0;
        for (int k = 1; k < kBins; ++k) {
          if (bin_n[k - 1]) { l.grow(bin_box[k - 1]); nl += bin_n[k - 1]; }
          const int nr = nright[k];
          if (!nl || !nr) continue;
          const double c = l.area() * nl + right[k].area() * nr;
          if (c < best) { best = c; best_k = k; best_axis = ax; }
        }
      }
      if (best_k > 0) {
        // leaf when splitting does not pay
        const double leaf_cost = bb.area() * n;
        if (n <= kBvhLeafMax && trav_cost * bb.area() + best >= leaf_cost) return leaf(b, n);
        axis = best_axis;
        ext = cb.hi[axis] - cb.lo[axis];
        const double lo = cb.lo[axis];
        mid = partition(b, e, [&](int i) { return bin_index(i, axis, lo, ext) < best_k; });
      }
    }
    if (mid <= b || mid >= e) {  // degenerate centroids or depth guard: median split
      mid = b + n / 2;
      sort_range(b, e, axis);
    }
    const int idx = (int)nodes.size();
    nodes.emplace_back();
    nodes[idx].axis = axis;
    Box lb, rb;
    const int32_t c0 = build(b, mid, depth + 1, &lb);
    const int32_t c1 = build(mid, e, depth + 1, &rb);
    BvhNode& nd = nodes[idx];
    nd.child[0] = c0;
    nd.child[1] = c1;
    for (int a = 0; a < 3; ++a) {
      nd.lo[0][a] = f32_down(lb.lo[a]); nd.hi[0][a] = f32_up(lb.hi[a]);
      nd.lo[1][a] = f32_down(rb.lo[a]); nd.hi[1][a] = f32_up(rb.hi[a]);
    }
    return idx;
  }

  int32_t leaf(int b, int n) { return -(1 + ((b << 7) | n)); }
  int bin_index(int i, int ax, double lo, double ex) const {
    const int k = (int)((cen[3 * i + ax] - lo) / ex * kBins);
    return std::min(std::max(k, 0), kBins - 1);
  }

  template <typename Pred>
  int partition(int b, int e, Pred left) {
    int i = b, j = e - 1;
    while (true) {
      while (i <= j && left(i)) ++i;
      while (i <= j && !left(j)) --j;
      if (i >= j) break;
      swap_items(i, j);
      ++i; --j;
    }
    return i;
  }
  void sort_range(int b, int e, int axis) {
    std::vector<int> idx(e - b);
    for (int i = 0; i < e - b; ++i) idx[i] = b + i;
    std::sort(idx.begin(), idx.end(), [&](int x, int y) {
      return cen[3 * x + axis] < cen[3 * y + axis] || (cen[3 * x + axis] == cen[3 * y + axis] && x < y);
    });
    std::vector<int> o2;
    std::vector<Box> b2;
    std::vector<double> c2;
    for (int i : idx) {
      o2.push_back(order[i]);
      b2.push_back(box[i]);
      c2.insert(c2.end(), &cen[3 * i], &cen[3 * i] + 3);
    }
    for (int i = b; i < e; ++i) {
      order[i] = o2[i - b];
      box[i] = b2[i - b];
      std::memcpy(&cen[3 * i], &c2[3 * (i - b)], 3 * sizeof(double));
    }
  }
  void swap_items(int i, int j) {
    std::swap(order[i], order[j]);
    std::swap(box[i], box[j]);
    for (int a = 0; a < 3; ++a) std::swap(cen[3 * i + a], cen[3 * j + a]);
  }
};

int tree_depth(const std::vector<BvhNode>& nodes, int32_t e) {
  if (e < 0) return 0;
  return 1 + std::max(tree_depth(nodes, nodes[e].child[0]), tree_depth(nodes, nodes[e].child[1]));
}

// The nodes renumbered for the treelet: the first kTreeletNodes in
// breadth-first order (root 0, then each level in turn), so that a prefix of
// the array is the top of the hierarchy (the global-memory image stages such a
// prefix in LDS), then each remaining subtree in depth-first order (its nodes
// contiguous, for the L2). The numbering changes neither the boxes nor the
// child order, so no traversal result changes.
constexpr size_t kTreeletNodes = 1536;
std::vector<BvhNode> treelet_order(const std::vector<BvhNode>& in) {
  if (in.empty()) return in;
  std::vector<int> order;
  order.reserve(in.size());
  std::vector<int> queue{0};
  size_t h = 0;
  for (; h < queue.size() && order.size() < kTreeletNodes; ++h) {
    order.push_back(queue[h]);
    for (int c = 0; c < 2; ++c)
      if (in[queue[h]].child[c] >= 0) queue.push_back(in[queue[h]].child[c]);
  }
  std::vector<int> stack;
  for (; h < queue.size(); ++h) {  // the frontier's subtrees, depth-first
    stack.assign(1, queue[h]);
    while (!stack.empty()) {
      const int e = stack.back();
      stack.pop_back();
      order.push_back(e);
      for (int c = 1; c >= 0; --c)
        if (in[e].child[c] >= 0) stack.push_back(in[e].child[c]);
    }
  }
  std::vector<int32_t> remap(in.size(), -1);
  for (size_t i = 0; i < order.size(); ++i) remap[order[i]] = (int32_t)i;
  std::vector<BvhNode> out(order.size());
  for (size_t i = 0; i < order.size(); ++i) {
    out[i] = in[order[i]];
    for (int c = 0; c < 2; ++c)
      if (out[i].child[c] >= 0) out[i].child[c] = remap[out[i].child[c]];
  }
  return out;
}

// The hierarchy over `boxes`; `order` receives the leaf order of the items.
std::vector<BvhNode> build_over_boxes(const std::vector<Box>& boxes, int leaf_size, double trav_cost, int* depth,
                                      std::vector<int>* order) {
  if (depth) *depth = 0;
  order->clear();
  std::vector<BvhNode> out;
  const int n = (int)boxes.size();
  if (n == 0) return out;
  // the leaf code stores the first index in 24 bits
  if (n >= (1 << 24)) return out;
  leaf_size = std::max(1, std::min(leaf_size, kBvhLeafMax));
  Builder bd{{}, boxes, {}, {}, leaf_size, trav_cost};
  bd.order.resize(n);
  bd.cen.resize(3 * n);
  for (int i = 0; i < n; ++i) {
    bd.order[i] = i;
    for (int a = 0; a < 3; ++a) bd.cen[3 * i + a] = 0.5 * (boxes[i].lo[a] + boxes[i].hi[a]);
  }
  bd.nodes.reserve(2 * n / std::max(1, leaf_size) + 2);
  Box all;
  const int32_t root = bd.build(0, n, 0, &all);
  if (root < 0) {  // a single leaf: wrap it in a root node (the traversal starts at node 0)
    BvhNode r{};
    r.child[0] = root;
    r.child[1] = kBvhEmpty;
    for (int a = 0; a < 3; ++a) { r.lo[0][a] = f32_down(all.lo[a]); r.hi[0][a] = f32_up(all.hi[a]); }
    bd.nodes.assign(1, r);
  }
  if (depth) *depth = tree_depth(bd.nodes, 0);  // kBvhEmpty < 0 counts as a leaf
  *order = bd.order;
  return treelet_order(bd.nodes);
}

template <typename R>
void apply_order(std::vector<R>& items, const std::vector<int>& order) {
  std::vector<R> out;
  out.reserve(order.size());
  for (int i : order) out.push_back(items[i]);
  items.swap(out);
}

// A = the 3x3 part of an inverse (rows 0-2), F = A^-1 by cofactors; returns
// |A|_inf * |F|_inf (the condition number), or +inf when A is singular.
double invert3(const double* m, double F[3][3]) {
  const double a[3][3] = {{m[0], m[1], m[2]}, {m[4], m[5], m[6]}, {m[8], m[9], m[10]}};
  const double c00 = a[1][1] * a[2][2] - a[1][2] * a[2][1];
  const double c01 = a[1][2] * a[2][0] - a[1][0] * a[2][2];
  const double c02 = a[1][0] * a[2][1] - a[1][1] * a[2][0];
  const double det = a[0][0] * c00 + a[0][1] * c01 + a[0][2] * c02;
  if (!(std::fabs(det) > 0.0) || !std::isfinite(det)) return INFINITY;
  F[0][0] = c00 / det;
  F[1][0] = c01 / det;
  F[2][0] = c02 / det;
  F[0][1] = (a[0][2] * a[2][1] - a[0][1] * a[2][2]) / det;
  F[1][1] = (a[0][0] * a[2][2] - a[0][2] * a[2][0]) / det;
  F[2][1] = (a[0][1] * a[2][0] - a[0][0] * a[2][1]) / det;
  F[0][2] = (a[0][1] * a[1][2] - a[0][2] * a[1][1]) / det;
  F[1][2] = (a[0][2] * a[1][0] - a[0][0] * a[1][2]) / det;
  F[2][2] = (a[0][0] * a[1][1] - a[0][1] * a[1][0]) / det;
  double na = 0.0, nf = 0.0;
  for (int r = 0; r < 3; ++r) {
    na = std::max(na, std::fabs(a[r][0]) + std::fabs(a[r][1]) + std::fabs(a[r][2]));
    nf = std::max(nf, std::fabs(F[r][0]) + std::fabs(F[r][1]) + std::fabs(F[r][2]));
  }
  const double k = na * nf;
  return std::isfinite(k) ? k : INFINITY;
}

}  // namespace

uint16_t f16_bits_down(double x) { return f16_bits(f16_floor(x)); }
uint16_t f16_bits_up(double x) { return f16_bits(-f16_floor(-x)); }

std::vector<BvhNode> build_sphere_bvh(std::vector<SphereDiag>& spheres, int leaf_size, int* depth, double trav_cost) {
  std::vector<Box> boxes(spheres.size());
  for (size_t i = 0; i < spheres.size(); ++i) boxes[i] = sphere_box(spheres[i]);
  std::vector<int> order;
  std::vector<BvhNode> nodes = build_over_boxes(boxes, leaf_size, trav_cost, depth, &order);
  if (!nodes.empty()) apply_order(spheres, order);
  return nodes;
}

std::vector<BvhPair> pair_layout(const std::vector<BvhNode>& nodes) {
  // the 16-bit child codes of the pair image (rt_layout.hpp BvhPair)
  auto code16 = [](int32_t c, bool* ok) -> int32_t {
    if (c == kBvhEmpty) return 0xFFFF;
    if (c >= 0) {
      if (c >= 0x8000) *ok = false;
      return c;
    }
    const int code = -(c + 1), first = code >> 7, cnt = code & 127;
    if (first >= 4095 || cnt < 1 || cnt > 8) *ok = false;
    return 0x8000 | (first << 3) | (cnt - 1);
  };
  bool ok = true;
  std::vector<BvhPair> out(nodes.size());
  for (size_t i = 0; i < nodes.size(); ++i) {
    const BvhNode& g = nodes[i];
    BvhPair& q = out[i];
    for (int a = 0; a < 3; ++a) {
      q.b[4 * a] = g.lo[0][a]; q.b[4 * a + 1] = g.lo[1][a]; q.b[4 * a + 2] = g.hi[0][a]; q.b[4 * a + 3] = g.hi[1][a];
    }
    q.child[0] = code16(g.child[0], &ok);
    q.child[1] = code16(g.child[1], &ok);
    q.axis = g.axis;
    q.pad = 0;
  }
  if (!ok) out.clear();  // not encodable: no pair image (the fast path reads the binary nodes from global memory)
  return out;
}

std::vector<BvhWide> wide_layout(const std::vector<BvhNode>& nodes, const std::vector<SphereDiag>& spheres,
                                 int* stack) {
  if (stack) *stack = 0;
  std::vector<BvhWide> tmp;
  if (nodes.empty()) return tmp;
  // a slot: a binary node (code >= 0) or a leaf (BvhNode's leaf code), with its box
  struct Slot {
    int32_t code;
    float lo[3], hi[3];
  };
  auto leaf_of = [](int32_t code, int* first, int* cnt) {
    const int c = -(code + 1);
    *first = c >> 7;
    *cnt = c & 127;
  };
  auto single = [](int k) { return (int32_t)-(1 + ((k << 7) | 1)); };
  // one record's own box, binary32 outward (what a one-record binary leaf stores)
  auto sphere_slot = [&](int k) {
    const Box b = sphere_box(spheres[k]);
    Slot s;
    s.code = single(k);
    for (int a = 0; a < 3; ++a) { s.lo[a] = f32_down(b.lo[a]); s.hi[a] = f32_up(b.hi[a]); }
    return s;
  };
  auto area = [](const Slot& s) {
    const double dx = (double)s.hi[0] - s.lo[0], dy = (double)s.hi[1] - s.lo[1], dz = (double)s.hi[2] - s.lo[2];
    return dx * dy + dy * dz + dz * dx;
  };
  auto children = [&](int n, std::vector<Slot>& out) {
    for (int c = 0; c < 2; ++c) {
      if (nodes[n].child[c] == kBvhEmpty) continue;
      Slot s;
      s.code = nodes[n].child[c];
      for (int a = 0; a < 3; ++a) { s.lo[a] = nodes[n].lo[c][a]; s.hi[a] = nodes[n].hi[c][a]; }
      out.push_back(s);
    }
  };
  std::vector<int> need;  // entries a near-first traversal keeps pending below each node
  bool ok = true;
  auto emit = [&](auto&& self, std::vector<Slot>& s) -> int {
    const int idx = (int)tmp.size();
    tmp.emplace_back(BvhWide{});
    need.push_back(0);
    int below = 0;
    for (size_t j = 0; j < 4; ++j) {
      int32_t c = 0xFFFF;
      float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      if (j < s.size()) {
        for (int a = 0; a < 3; ++a) { lo[a] = s[j].lo[a]; hi[a] = s[j].hi[a]; }
        int first = 0, cnt = 0;
        if (s[j].code >= 0) {
          std::vector<Slot> sub;
          children(s[j].code, sub);
          c = self(self, sub);
        } else if (leaf_of(s[j].code, &first, &cnt), cnt == 1) {
          if (first >= 0x7FFF) ok = false;
          c = 0x8000 | first;
        } else {
          // a record range the binary tree keeps in one leaf: nodes of up to four
          // parts, down to single records
          std::vector<Slot> sub;
          const int per = (cnt + 3) / 4;
          for (int p = first; p < first + cnt; p += per) {
            const int m = std::min(per, first + cnt - p);
            if (m == 1) { sub.push_back(sphere_slot(p)); continue; }
            Slot r = sphere_slot(p);
            r.code = (int32_t)-(1 + ((p << 7) | m));
            for (int k = p + 1; k < p + m; ++k) {
              const Slot q = sphere_slot(k);
              for (int a = 0; a < 3; ++a) { r.lo[a] = std::min(r.lo[a], q.lo[a]); r.hi[a] = std::max(r.hi[a], q.hi[a]); }
            }
            sub.push_back(r);
          }
          c = self(self, sub);
        }
        if (c < 0x8000) below = std::max(below, need[c]);
      }
      BvhWide& w = tmp[idx];
      w.child[j] = (uint16_t)c;
      for (int a = 0; a < 3; ++a) { w.lo[a][j] = lo[a]; w.hi[a][j] = hi[a]; }
    }
    need[idx] = (int)s.size() - 1 + below;
    return idx;
  };
  // a node's slots: its binary children, opening the largest-area one (a
  // binary node, or a leaf of several records that fits whole) until four
  auto open = [&](std::vector<Slot>& s) {
    while (s.size() < 4) {
      int best = -1;
      for (size_t j = 0; j < s.size(); ++j) {
        int first, cnt = 1;
        if (s[j].code < 0) leaf_of(s[j].code, &first, &cnt);
        const bool can = s[j].code >= 0 || (cnt > 1 && s.size() - 1 + (size_t)cnt <= 4);
        if (can && (best < 0 || area(s[j]) > area(s[best]))) best = (int)j;
      }
      if (best < 0) break;
      const Slot o = s[best];
      s.erase(s.begin() + best);
      if (o.code >= 0) {
        children(o.code, s);
      } else {
        int first, cnt;
        leaf_of(o.code, &first, &cnt);
        for (int k = first; k < first + cnt; ++k) s.push_back(sphere_slot(k));
      }
    }
  };
  auto build = [&](auto&& self, std::vector<Slot>& s) -> int {
    open(s);
    return emit(self, s);
  };
  {
    std::vector<Slot> root;
    children(0, root);
    build(build, root);
  }
  if (!ok || tmp.size() >= 0x8000) return {};
  if (stack) *stack = need[0];
  // renumber: breadth-first for the first kTreeletNodes nodes, then each
  // remaining subtree depth-first (as treelet_order does for the binary nodes)
  std::vector<int> order{0};
  size_t h = 0;
  for (; h < order.size() && order.size() < kTreeletNodes; ++h)
    for (int j = 0; j < 4; ++j)
      if (tmp[order[h]].child[j] < 0x8000) order.push_back(tmp[order[h]].child[j]);
  std::vector<int> frontier(order.begin() + (long)h, order.end()), st;
  order.resize(h);
  for (int f : frontier) {
    st.assign(1, f);
    while (!st.empty()) {
      const int e = st.back();
      st.pop_back();
      order.push_back(e);
      for (int j = 3; j >= 0; --j)
        if (tmp[e].child[j] < 0x8000) st.push_back(tmp[e].child[j]);
    }
  }
  std::vector<int32_t> remap(tmp.size(), -1);
  for (size_t i = 0; i < order.size(); ++i) remap[order[i]] = (int32_t)i;
  std::vector<BvhWide> out(order.size());
  for (size_t i = 0; i < order.size(); ++i) {
    out[i] = tmp[order[i]];
    for (int j = 0; j < 4; ++j)
      if (out[i].child[j] < 0x8000) out[i].child[j] = remap[out[i].child[j]];
  }
  return out;
}

std::vector<BvhWide16> wide16_layout(const std::vector<BvhWide>& w) {
  std::vector<BvhWide16> out(w.size());
  for (size_t i = 0; i < w.size(); ++i) {
    for (int a = 0; a < 3; ++a)
      for (int j = 0; j < 4; ++j) {
        out[i].lo[a][j] = f16_bits_down(w[i].lo[a][j]);
        out[i].hi[a][j] = f16_bits_up(w[i].hi[a][j]);
      }
    for (int j = 0; j < 4; ++j) out[i].child[j] = w[i].child[j];
  }
  return out;
}

// the padded world box of a record's local region [L, U] under its stored
// inverse (false: too ill-conditioned for the padding argument)
static bool region_box(const OtherRec& r, const double L[3], const double U[3], double lo[3], double hi[3]) {
  double F[3][3];
  const double cond = invert3(r.m, F);
  if (!(cond <= 1e6)) return false;  // too ill-conditioned for the padding argument
  const double b[3] = {r.m[3], r.m[7], r.m[11]};
  for (int i = 0; i < 3; ++i) {
    // world point p = F (q - b) for a local point q of the record's region
    double c = 0.0, h = 0.0;
    for (int j = 0; j < 3; ++j) {
      c += F[i][j] * (0.5 * (L[j] + U[j]) - b[j]);
      h += r.kind == 0 ? F[i][j] * F[i][j] : std::fabs(F[i][j]) * 0.5 * (U[j] - L[j]);
    }
    if (r.kind == 0) h = std::sqrt(h);  // the ellipsoid's extent along axis i
    h *= 1.0 + 1e-12;                   // the rounding of F, c and h themselves
    if (!std::isfinite(c) || !std::isfinite(h)) return false;
    pad_axis(c - h, c + h, &lo[i], &hi[i]);
  }
  return true;
}

bool other_box(const OtherRec& r, double lo[3], double hi[3]) {
  // cones go to the line hierarchy (line_box): their a ~ 0 branch pushes t =
  // -c / 2.0 * b (cone.rs:104), a root that need not lie on the cone at all
  if (r.kind != 0 && r.kind != 2 && r.kind != 3) return false;
  double L[3] = {-1.0, -1.0, -1.0}, U[3] = {1.0, 1.0, 1.0};
  if (r.kind == 3) {  // cylinder: culled here only when closed, with finite caps' planes
    // An OPEN tube goes to the line hierarchy: the culling argument here needs
    // "an odd number of t < 0 roots => the origin lies inside the box"
    // (DESIGN.md §5.2), true for closed convex solids only. A backward line can
    // cross one wall of an open tube within [min, max] and leave through the
    // open end, so the tube is a `containers` entry (intersection.rs:63-90) for
    // a ray whose [0, t_hi] never meets its box.
    if (!r.closed) return false;
    if (!std::isfinite(r.minimum) || !std::isfinite(r.maximum) || !(r.minimum <= r.maximum)) return false;
    L[1] = r.minimum;
    U[1] = r.maximum;
  }
  return region_box(r, L, U, lo, hi);
}

bool line_box(const QuadRec& r, double lo[3], double hi[3]) {
  if (!(r.kind == 4 || (r.kind == 3 && !r.closed))) return false;
  if (!std::isfinite(r.minimum) || !std::isfinite(r.maximum) || !(r.minimum <= r.maximum)) return false;
  // the reference's own boxes: cylinder.rs (radius 1), cone.rs:27-46 (radius max(|min|, |max|))
  const double w = r.kind == 4 ? std::max(std::fabs(r.minimum), std::fabs(r.maximum)) : 1.0;
  const double L[3] = {-w, r.minimum, -w}, U[3] = {w, r.maximum, w};
  return region_box(r, L, U, lo, hi);
}

std::vector<BvhNode> build_other_bvh(std::vector<OtherRec>& recs, int leaf_size, int* depth, double trav_cost) {
  std::vector<Box> boxes(recs.size());
  for (size_t i = 0; i < recs.size(); ++i)
    if (!other_box(recs[i], boxes[i].lo, boxes[i].hi)) return {};  // the caller passes bounded records only
  std::vector<int> order;
  std::vector<BvhNode> nodes = build_over_boxes(boxes, leaf_size, trav_cost, depth, &order);
  if (!nodes.empty()) apply_order(recs, order);
  return nodes;
}

std::vector<BvhNode> build_line_bvh(std::vector<QuadRec>& recs, std::vector<ConeCluster>* clusters,
                                    std::vector<int32_t>* members, int* depth) {
  clusters->clear();
  members->clear();
  std::vector<Box> boxes(recs.size());
  for (size_t i = 0; i < recs.size(); ++i)
    if (!line_box(recs[i], boxes[i].lo, boxes[i].hi)) return {};
  std::vector<int> order;
  // one record per leaf where the builder can split (line_trace tests each record of a leaf)
  std::vector<BvhNode> nodes = build_over_boxes(boxes, 1, 1.0, depth, &order);
  if (nodes.empty()) return nodes;
  apply_order(recs, order);
  // per cone: Q = m0 m0^T - m1 m1^T + m2 m2^T (m_k: row k of the inverse's 3x3
  // part; a(d) = d^T Q d exactly), and W = sum_k (sum_j |m_kj|)^2: the
  // reference's a (object direction m d, then dx*dx - dy*dy + dz*dz, every
  // operation rounded) is within 16 u W dm^2 of d^T Q d (u = 2^-53)
  const double u = 0x1p-53;
  const int ij[6][2] = {{0, 0}, {1, 1}, {2, 2}, {0, 1}, {0, 2}, {1, 2}};
  std::map<std::array<double, 6>, std::vector<int>> by_q;  // cones of one (bitwise) Q, in record order
  std::map<std::array<double, 6>, double> w_max;
  for (size_t k = 0; k < recs.size(); ++k) {
    if (recs[k].kind != 4) continue;
    const double* m = recs[k].m;
    const double R[3][3] = {{m[0], m[1], m[2]}, {m[4], m[5], m[6]}, {m[8], m[9], m[10]}};
    std::array<double, 6> q;
    for (int e = 0; e < 6; ++e)
      q[e] = R[0][ij[e][0]] * R[0][ij[e][1]] - R[1][ij[e][0]] * R[1][ij[e][1]] + R[2][ij[e][0]] * R[2][ij[e][1]];
    double w = 0.0;
    for (int r = 0; r < 3; ++r) {
      const double s = std::fabs(R[r][0]) + std::fabs(R[r][1]) + std::fabs(R[r][2]);
      w += s * s;
    }
    by_q[q].push_back((int)k);
    double& wm = w_max[q];
    wm = std::max(wm, w);
  }
  for (const auto& [q, ks] : by_q) {
    ConeCluster c{};
    for (int e = 0; e < 6; ++e) c.q[e] = q[e];
    const double aq = std::fabs(q[0]) + std::fabs(q[1]) + std::fabs(q[2]) +
                      2.0 * (std::fabs(q[3]) + std::fabs(q[4]) + std::fabs(q[5]));  // sum of |Q| over nine entries
    // the reference's rounding (16 u W), the device's g (8 u |Q|), this host
    // arithmetic's Q (1e-12 |Q|), then a relative margin
    c.r = (16.0 * u * w_max.at(q) + 8.0 * u * aq + 1e-12 * aq) * (1.0 + 1e-9);
    if (!std::isfinite(c.r)) return {};
    c.first = (int32_t)members->size();
    c.count = (int32_t)ks.size();
    members->insert(members->end(), ks.begin(), ks.end());
    clusters->push_back(c);
  }
  return nodes;
}

// ------------------------------------------------------------ light buffer
// See rt_layout.hpp (LbCell) and DESIGN.md "Light buffer" for the argument.
// Margins: the query (binary32, from the binary64 shadow-ray vector) lands
// within ~1e-6 (cube-map coordinate units) of the exact direction of any
// root point at distance >= r0 from the light while |light - o| <= 2^24 r0;
// the pyramid of a face is relaxed by kLbEta and every coordinate range is
// widened by kLbMargin, both 1e-5.
namespace {
constexpr double kLbEta = 1e-5, kLbMargin = 1e-5;

// distance from the origin to the box, 0 when it contains the origin
double box_dist0(const double* lo, const double* hi) {
  double s = 0.0;
  for (int a = 0; a < 3; ++a) {
    const double g = lo[a] > 0.0 ? lo[a] : hi[a] < 0.0 ? -hi[a] : 0.0;
    s += g * g;
  }
  return std::sqrt(s);
}
double min_abs(double lo, double hi) { return lo > 0.0 ? lo : hi < 0.0 ? -hi : 0.0; }
int lb_cell_index(double x, int R) {  // x in [-1, 1]
  const int i = (int)std::floor((x + 1.0) * 0.5 * R);
  return std::max(0, std::min(R - 1, i));
}
}  // namespace

LightBuffer build_light_buffer(const std::vector<SphereDiag>& sph, const std::vector<LightRec>& lights, int R) {
  LightBuffer lb;
  const int n = (int)sph.size();
  if (n == 0 || n >= 0xFFFF || R < 1 || lights.empty()) return lb;
  lb.res = R;
  const size_t per = (size_t)6 * R * R;
  lb.cells.assign(lights.size() * per, LbCell{0, 0, 0, 0});
  lb.delta.assign(lights.size() * (size_t)n, 0.0f);
  lb.limit.assign(lights.size(), -1.0f);
  std::vector<std::array<double, 6>> rel(n);
  std::vector<double> delta(n);
  std::vector<char> finite(n), caster(n), near(n);
  for (size_t l = 0; l < lights.size(); ++l) {
    const double* L = lights[l].pos;
    if (!(std::isfinite(L[0]) && std::isfinite(L[1]) && std::isfinite(L[2]))) continue;  // limit -1: exhaustive
    double dmax = 0.0;
    for (int i = 0; i < n; ++i) {
      caster[i] = (sph[i].meta & 1) != 0;
      const Box b = sphere_box(sph[i]);
      bool fin = true;
      for (int a = 0; a < 3; ++a) {
        rel[i][a] = b.lo[a] - L[a];
        rel[i][3 + a] = b.hi[a] - L[a];
        fin = fin && std::isfinite(rel[i][a]) && std::isfinite(rel[i][3 + a]);
      }
      finite[i] = fin;
      delta[i] = fin ? box_dist0(&rel[i][0], &rel[i][3]) * (1.0 - 1e-9) : 0.0;
      if (caster[i] && fin) dmax = std::max(dmax, delta[i]);
      lb.delta[l * n + i] = f32_down(delta[i]);
    }
    // records whose box comes within 1e-3 of the farthest box's distance are
    // listed in every cell; r0 = the nearest of the others
    const double r_near = 1e-3 * dmax;
    double r0 = INFINITY;
    for (int i = 0; i < n; ++i) {
      near[i] = 0;
      if (!caster[i]) continue;
      near[i] = !finite[i] || delta[i] < r_near || delta[i] == 0.0;
      if (!near[i]) r0 = std::min(r0, delta[i]);
    }
    lb.limit[l] = std::isfinite(r0) ? f32_down(std::min(0x1p24 * r0, 1e30)) : 1e30f;
    auto face_rect = [&](int i, int f, int* r) {
      r[0] = -1;
      const int a = f >> 1, bx = (a + 1) % 3, cx = (a + 2) % 3;
      const double s = (f & 1) ? -1.0 : 1.0;
      const double* lo = &rel[i][0];
      const double* hi = &rel[i][3];
      const double A_lo = s > 0 ? lo[a] : -hi[a], A_hi = s > 0 ? hi[a] : -lo[a];
      if (!(A_hi > 0.0)) return;
      const double a_min = std::max(A_lo, std::max(min_abs(lo[bx], hi[bx]), min_abs(lo[cx], hi[cx])) / (1.0 + kLbEta));
      if (a_min > A_hi) return;
      double u_lo = -1.0, u_hi = 1.0, v_lo = -1.0, v_hi = 1.0;
      if (a_min > 0.0) {
        u_lo = std::min(lo[bx] / a_min, lo[bx] / A_hi) - kLbMargin;
        u_hi = std::max(hi[bx] / a_min, hi[bx] / A_hi) + kLbMargin;
        v_lo = std::min(lo[cx] / a_min, lo[cx] / A_hi) - kLbMargin;
        v_hi = std::max(hi[cx] / a_min, hi[cx] / A_hi) + kLbMargin;
      }
      r[0] = lb_cell_index(std::max(-1.0, std::min(1.0, u_lo)), R);
      r[1] = lb_cell_index(std::max(-1.0, std::min(1.0, u_hi)), R);
      r[2] = lb_cell_index(std::max(-1.0, std::min(1.0, v_lo)), R);
      r[3] = lb_cell_index(std::max(-1.0, std::min(1.0, v_hi)), R);
    };
    // the lists as one flat array (counts, offsets, fill; each face's cells get
    // entries only from that face's rectangles, so the six faces are built in
    // parallel, each in increasing record order), then every cell sorted and
    // encoded in parallel over contiguous blocks of cells
    // (small maps: one thread, the threads would cost more than they save)
    const bool par = per >= ((size_t)1 << 17);
    const unsigned nt = par ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
    std::vector<std::array<int, 4>> rects((size_t)n * 6);
    std::vector<uint32_t> cnt(per + 1, 0);
    auto for_faces = [&](auto&& fn) {
      if (!par) {
        for (int f = 0; f < 6; ++f) fn(f);
        return;
      }
      std::vector<std::thread> th;
      for (int f = 0; f < 6; ++f) th.emplace_back(fn, f);
      for (std::thread& t : th) t.join();
    };
    for_faces([&](int f) {
      for (int i = 0; i < n; ++i) {
        int* r = rects[(size_t)i * 6 + f].data();
        r[0] = -1;
        if (!caster[i]) continue;
        if (near[i]) { r[0] = 0; r[1] = R - 1; r[2] = 0; r[3] = R - 1; }
        else face_rect(i, f, r);
        if (r[0] < 0) continue;
        for (int j = r[2]; j <= r[3]; ++j)
          for (int k = r[0]; k <= r[1]; ++k) ++cnt[(size_t)f * R * R + (size_t)j * R + k];
      }
    });
    std::vector<uint64_t> off(per + 1, 0);
    for (size_t c = 0; c < per; ++c) off[c + 1] = off[c] + cnt[c];
    std::vector<uint16_t> items(off[per]);
    for_faces([&](int f) {
      std::vector<uint64_t> pos(off.begin() + (long)f * R * R, off.begin() + (long)(f + 1) * R * R);
      for (int i = 0; i < n; ++i) {
        const int* r = rects[(size_t)i * 6 + f].data();
        if (r[0] < 0) continue;
        for (int j = r[2]; j <= r[3]; ++j)
          for (int k = r[0]; k <= r[1]; ++k) items[pos[(size_t)j * R + k]++] = (uint16_t)i;
      }
    });
    // entries past the inline ones go to lb.ov, cell by cell
    std::vector<uint64_t> ovo(per + 1, 0);
    for (size_t c = 0; c < per; ++c) ovo[c + 1] = ovo[c] + (cnt[c] > (uint32_t)kLbInline ? cnt[c] - kLbInline : 0);
    const size_t ov0 = lb.ov.size();
    lb.ov.resize(ov0 + ovo[per]);
    const float* dl = &lb.delta[l * n];
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {  // (contiguous blocks of cells: no two threads share a line)
        for (size_t c = per * t / nt; c < per * (t + 1) / nt; ++c) {
          uint16_t* v = items.data() + off[c];
          const size_t m = cnt[c];
          std::sort(v, v + m, [&](uint16_t x, uint16_t y) { return dl[x] < dl[y] || (dl[x] == dl[y] && x < y); });
          uint16_t in[kLbInline] = {0, 0, 0, 0, 0};
          for (size_t k = 0; k < m && k < (size_t)kLbInline; ++k) in[k] = v[k];
          LbCell& cell = lb.cells[l * per + c];
          cell.w0 = (uint32_t)std::min<size_t>(m, 0xFFFF) | (uint32_t)in[0] << 16;
          cell.w1 = in[1] | (uint32_t)in[2] << 16;
          cell.w2 = in[3] | (uint32_t)in[4] << 16;
          cell.ov = (uint32_t)(ov0 + ovo[c]);
          for (size_t k = kLbInline; k < m; ++k) lb.ov[ov0 + ovo[c] + (k - kLbInline)] = v[k];
        }
      });
    for (std::thread& t : th) t.join();
    lb.n_items += off[per];
  }
  return lb;
}

}  // namespace rtamd
