// rt_persist.hpp — the persistent frame kernel (DESIGN.md §5.1 "Persistent
// frames"): ONE launch renders a whole frame (or shard, or ray batch) through
// every recursion depth of `World::color_at` (world.rs:70-81).
//
// Each workgroup (one per CU: the LDS scene image) stages the image once and
// then its 16 waves pull work until the frame is done:
//   - a chunk of 64 camera rays (a "tree": the recursion trees of 64 root
//     rays), taken from a per-frame counter shared by all workgroups, or
//   - up to 64 queued child rays from the workgroup's own ring.
// A wave traces its 64 rays (closest hit, prepare_computations, every light's
// shadow ray and lighting()), appends the reflected / refracted children to
// the ring, and writes a PsParent record (and an entry in the tree's list of
// that depth) for every node with children. A node without children knows its
// colour at once and writes it into its parent's record. The wave whose ray
// finishes a tree (an LDS count of the tree's unfinished rays) evaluates
// shade_hit's expression (world.rs:58-67) for the tree's nodes with children,
// deepest depth first, and writes the roots' colours to the canvas.
//
// Every hand-off stays inside one workgroup (one CU): ring slots and parent
// records are written with non-temporal stores (kept in the XCD's L2), made
// visible by `s_waitcnt vmcnt(0)` before the LDS counter that publishes them,
// and read with non-temporal loads (served by the L2, never a stale L1 line).
// No workgroup ever waits for another one, so the grid needs no co-residency.
//
// Parent records are addressed by position, not allocated: tree t, root ray
// (pixel) p, heap node n of that root's binary recursion tree (children of n:
// 2n+1 reflected, 2n+2 refracted). Node n lies at depth floor(log2(n+1)), so
// max_depth <= kPsMaxDepth (heap nodes < 1024); deeper renders take the
// generation pipeline (rt_wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.hpp"

namespace rtamd {

constexpr unsigned kPsMaxDepth = 8;      // heap node ids of depth <= 8 fit 10 bits
constexpr unsigned kPsMaxTrees = 32;     // tree slots per workgroup (one LDS bitmask)
constexpr unsigned kPsSpare = 1024;      // ring slots claimed but not yet read (16 waves x 64)
constexpr size_t kPsSchedBytes = 1536;   // LDS of the scheduler state (PsSched), beside the scene image
// device memory of a workspace's trees (parents + rings) at the largest grid:
// sets the tree slots per workgroup for deep recursion (C5, depth 8: 14)
constexpr size_t kPsBudget = (size_t)12 << 30;

struct alignas(64) PsRay {  // 64 B: one queued child ray
  double o[3];
  double d[3];
  uint32_t id;  // tree << 16 | root << 10 | heap node
  uint32_t pad[3];
};
static_assert(sizeof(PsRay) == 64, "PsRay must stay 64 B");

struct alignas(128) PsParent {  // 128 B (one L2 line): a node with children
  double surface[3];  // the lighting sum over the lights (world.rs:41-56)
  double schlick;     // Computations::schlick (only read when reflective && transparent)
  double refl[3];     // the reflected child's colour (color_at of the child ray)
  double pad0;
  double refr[3];     // the refracted child's colour
  double pad1;
  int32_t obj;
  uint32_t kids;     // bit 0: reflected child, bit 1: refracted child
  uint32_t n_kids;
  uint32_t pad2[5];
};
static_assert(sizeof(PsParent) == 128, "PsParent must stay 128 B");

// Per-frame work counters of a workspace: the camera-chunk counter of each
// class (blocks are dealt round-robin to the XCDs: class = block % classes),
// 128 B apart, and the count of finished workgroups (the last one zeroes all
// of them for the next frame on the workspace).
constexpr unsigned kPsClasses = 8;
constexpr unsigned kPsCtrStride = 32;
struct PsCounters {
  unsigned chunk[kPsClasses * kPsCtrStride];
  unsigned done;
  unsigned pad[kPsCtrStride - 1];
};

struct PsArgs {
  PsRay* rings;        // grid x q_cap
  PsParent* parents;   // grid x trees x 64 x n_int
  uint16_t* lists;     // grid x trees x 64 x n_int: per tree and depth, (root << 10 | node) of its nodes with children
  PsCounters* ctr;
  void* cnt;           // WfCounters (counted launches)
  double* out;         // camera, aa == 1: the shard canvas (row-major); else root colours by root index
  const double* in_rays;  // batch mode: n0 x 6 doubles
  int* fault;          // host-mapped: a wait exceeded its time bound (the frame is incomplete)
  unsigned q_cap, n_int, trees;
  unsigned n0, max_depth;
  unsigned camera_mode, aa, rows, row_block, shard, n_shards;
  unsigned use_lb, lds_flags, n_top, skip_shadow, count;
  unsigned policy;  // WfTuning::ps_policy: 0 = queued rays before an idle wave; 1 = a partial chunk only when no other wave can add to it
};

// Launchers (rt_persist.hip, one object per image class): the LDS image
// (pair layout, image 14) and the global-memory images (3: LDS stack and
// treelet, 1: scratch stack). `grid` workgroups of kTraceBlock threads, `lds`
// dynamic LDS bytes; e0 / e1 (may be null) are recorded by the dispatch itself.
hipError_t ps_launch_lds(const DevScene& sc, const DevCamera& cam, const PsArgs& a, bool quads, bool tally,
                         unsigned grid, size_t lds, hipStream_t st, hipEvent_t e0, hipEvent_t e1);
hipError_t ps_launch_global(const DevScene& sc, const DevCamera& cam, const PsArgs& a, int image, bool quads,
                            bool tally, unsigned grid, size_t lds, hipStream_t st, hipEvent_t e0, hipEvent_t e1);

}  // namespace rtamd
