// rt_bvh.hpp — host-side BVH over the SphereDiag records (see rt_layout.hpp).
#pragma once
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

}  // namespace rtamd
