// rt_kernels.hpp — host-visible launch interface of the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.hpp"

namespace rtamd {

constexpr int kMaxDepth = 64;  // deepest recursion a launch supports
constexpr int kDefaultWaves = 3;  // min waves/SIMD the render kernel is compiled for

struct RenderArgs {
  double* out;              // device: n_tasks * 3 doubles
  const double* rays;       // device: n_tasks * 6 doubles (batch) or nullptr (camera)
  unsigned* counter;        // device work counter, zeroed before the launch
  DevStats* stats;          // device counters (accumulated) or nullptr
  uint32_t n_tasks;         // pixels of this shard (or rays)
  uint32_t max_depth;       // MAX_RECURSION_DEPTH (world.rs:16) / `remaining`
  uint32_t row_block, shard, n_shards;
  int grid_cap;             // 0 = occupancy-limited persistent grid
  int waves;                // occupancy variant (0 = kDefaultWaves); tuning knob
};

hipError_t launch_render(const DevScene& sc, const DevCamera& cam, const RenderArgs& args,
                         hipStream_t stream);
hipError_t launch_hit(const DevScene& sc, const double* d_rays, int n, double* d_out, hipStream_t s);
hipError_t launch_shadow(const DevScene& sc, const double* d_pts, int n, int light, uint8_t* d_out,
                         hipStream_t s);

}  // namespace rtamd
