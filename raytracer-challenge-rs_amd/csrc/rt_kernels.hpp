// rt_kernels.hpp — host-visible launch interface of the batch kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.hpp"

namespace rtamd {

constexpr int kMaxDepth = 64;  // deepest recursion (max_depth / remaining) a render supports

hipError_t launch_hit(const DevScene& sc, const double* d_rays, int n, double* d_out, hipStream_t s);
// the specular pow (rt_pow.hpp) of n pairs (test hook)
hipError_t launch_pow(const double* d_x, const double* d_y, int n, double* d_out, hipStream_t s);
hipError_t launch_shadow(const DevScene& sc, const double* d_pts, int n, int light, uint8_t* d_out,
                         hipStream_t s);

}  // namespace rtamd
