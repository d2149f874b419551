// rt_bvh.hpp — host-side BVHs over the bounded records and the light buffer (see rt_layout.hpp).
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

// The nodes in the pair layout of the per-lane traversal (rt_layout.hpp BvhPair).
std::vector<BvhPair> pair_layout(const std::vector<BvhNode>& nodes);

// The hierarchy collapsed to four children per node (rt_layout.hpp BvhWide)
// over the records in leaf order (`spheres`, as build_sphere_bvh left them):
// each node takes its binary children and opens the one of largest box area
// (a binary node, or a leaf of several records that fits whole) until it
// holds four; every leaf of the result is one record (code 0x8000 | index).
// Node 0 is the root; the first nodes are in breadth-first order (a prefix is
// the top of the tree, for an LDS treelet). `stack` receives the most entries
// a near-first traversal keeps pending. Empty when the 16-bit codes cannot
// index the nodes or records.
std::vector<BvhWide> wide_layout(const std::vector<BvhNode>& nodes, const std::vector<SphereDiag>& spheres,
                                 int* stack);

// the global-memory copy of a four-wide image: its boxes rounded outward to binary16
std::vector<BvhWide16> wide16_layout(const std::vector<BvhWide>& w);
// binary16 bit patterns rounded outward (BvhWide16 boxes)
uint16_t f16_bits_down(double x);
uint16_t f16_bits_up(double x);

// The other bounded records (general-transform spheres, cubes, closed
// cylinders with finite caps; rt_layout.hpp OtherRec): other_box gives the
// padded world box of one (false for a cone, an open or unbounded cylinder,
// an ill-conditioned transform: the line hierarchy or the exhaustive loop
// takes those). build_other_bvh builds
// the hierarchy over records that all have one (reordered in place into leaf
// order); empty when there are none.
bool other_box(const OtherRec& r, double lo[3], double hi[3]);
std::vector<BvhNode> build_other_bvh(std::vector<OtherRec>& recs, int leaf_size, int* depth = nullptr,
                                     double trav_cost = 1.0);

// The line hierarchy (rt_layout.hpp ConeCluster): line_box
// gives the padded world box of an open tube or a cone with finite bounds
// (false for any other record, or an ill-conditioned transform);
// build_line_bvh builds the hierarchy over records that all have one, leaves
// of one record where the builder can split (reordered in place into leaf
// order), and the cones' clusters (cones of one direction quadratic, their
// members' indices into `recs` in `members`); empty when there are none.
bool line_box(const QuadRec& r, double lo[3], double hi[3]);
std::vector<BvhNode> build_line_bvh(std::vector<QuadRec>& recs, std::vector<ConeCluster>* clusters,
                                    std::vector<int32_t>* members, int* depth = nullptr);

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
