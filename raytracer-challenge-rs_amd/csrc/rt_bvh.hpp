// rt_bvh.hpp — host-side BVH over the SphereDiag records (see rt_layout.hpp).
#pragma once
#include <stddef.h>
#include <vector>

#include "rt_layout.hpp"

namespace rtamd {

// Builds the hierarchy over `spheres` (reordered in place into leaf order;
// `meta` keeps each record's object index, so keys and results do not depend
// on the order). Boxes are the exact world-space extent of each record's
// unit sphere under its stored inverse, padded outward (conservative
// culling: DESIGN.md "Exact culling"). Returns the node array (root = 0),
// empty when there are no spheres.
// `depth` receives the most far children a near-first traversal keeps
// pending (the number of internal nodes on the longest root-leaf path).
// `trav_cost`: SAH cost of a node visit relative to one sphere test.
std::vector<BvhNode> build_sphere_bvh(std::vector<SphereDiag>& spheres, int leaf_size, int* depth = nullptr,
                                      double trav_cost = 1.0);

// Collapses the binary hierarchy into four-wide nodes (root = 0): each node
// repeatedly opens its largest-area internal child until it holds four
// children. Boxes and leaf codes are copied unchanged, so the four-wide
// traversal culls exactly what the binary one may cull. `stack` receives the
// most entries a nearest-first traversal keeps pending (on a root-leaf path,
// the sum of (children - 1) over its nodes). `code16` tells whether every
// child fits BvhNode4::code.
std::vector<BvhNode4> collapse_bvh4(const std::vector<BvhNode>& bin, int* stack = nullptr, bool* code16 = nullptr);

// Fills BvhNode::code16 of every node; returns whether every child fits the
// 16-bit code (else the 16-bit traversal is not used).
bool fill_code16(std::vector<BvhNode>& bin);

// Light buffer over the shadow-casting records, one cube map of R x R cells
// per face per light (rt_layout.hpp LbCell; DESIGN.md "Light buffer").
// Empty (cells.size() == 0) when there are no records, or 65535 or more.
struct LightBuffer {
  int res = 0;
  size_t n_items = 0;
  std::vector<LbCell> cells;    // n_lights * 6R^2
  std::vector<uint16_t> ov;     // list entries past the inline ones
  std::vector<float> delta;     // n_lights * n_records
  std::vector<float> limit;     // per light
};
LightBuffer build_light_buffer(const std::vector<SphereDiag>& spheres, const std::vector<LightRec>& lights, int R);

}  // namespace rtamd
