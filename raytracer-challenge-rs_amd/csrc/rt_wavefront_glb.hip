// rt_wavefront_glb.hip — the fast path's launches over the global-memory
// scene images (LANE 3: the treelet and the stack in LDS; LANE 1: the stack in
// LDS; LANE 4: the four-wide global image). Its own code object, compiled
// without the AMDGPU register-pressure trackers (Makefile), which help the LDS
// image (C3) and cost the global images (C5) ~2 %.
#include "rt_wf_device.hpp"

#include <hip/hip_ext.h>

#pragma clang fp contract(off)

namespace rtamd {

template <typename K>
static int occupancy_grid(K kern, int block, size_t lds, unsigned n) {
  int dev = 0, n_cu = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  long long want = ((long long)n + block - 1) / block;
  long long cap = (long long)n_cu * per_cu;
  long long g = std::min(want, cap);
  return (int)std::max(g, 1LL);
}
template <bool QUADS, int LANE, bool TALLY, bool CAM>
static hipError_t launch_glb(const DevScene& sc, const DevCamera& cam, const WfArgs& a, size_t dyn, unsigned n,
                             hipStream_t stream, int block, hipEvent_t e0, hipEvent_t e1) {
  auto kern = wf_trace_fused<false, QUADS, LANE, TALLY, CAM>;
  if (dyn > 0) WF_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
  const dim3 grid(occupancy_grid(kern, block, dyn, n));
  if (e0) hipExtLaunchKernelGGL(kern, grid, dim3(block), dyn, stream, e0, e1, 0, sc, cam, a);
  else hipLaunchKernelGGL(kern, grid, dim3(block), dyn, stream, sc, cam, a);
  return hipGetLastError();
}
template <int LANE>
static hipError_t launch_glb_lane(bool quads, bool tally, bool cam_rays, const DevScene& sc, const DevCamera& cam,
                                  const WfArgs& a, size_t dyn, unsigned n, hipStream_t stream, int block, hipEvent_t e0,
                                  hipEvent_t e1) {
#define RT_GLB(Q, T, C) launch_glb<Q, LANE, T, C>(sc, cam, a, dyn, n, stream, block, e0, e1)
  if (cam_rays) {
    if (quads) return tally ? RT_GLB(true, true, true) : RT_GLB(true, false, true);
    return tally ? RT_GLB(false, true, true) : RT_GLB(false, false, true);
  }
  if (quads) return tally ? RT_GLB(true, true, false) : RT_GLB(true, false, false);
  return tally ? RT_GLB(false, true, false) : RT_GLB(false, false, false);
#undef RT_GLB
}
hipError_t wf_launch_global(int lane, bool quads, bool tally, bool cam_rays, const DevScene& sc, const DevCamera& cam,
                            const WfArgs& a, size_t dyn, unsigned n, hipStream_t stream, int block, hipEvent_t e0,
                            hipEvent_t e1) {
  if (lane == 3) return launch_glb_lane<3>(quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, e0, e1);
  if (lane == 1) return launch_glb_lane<1>(quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, e0, e1);
  if (lane == 4) return launch_glb_lane<4>(quads, tally, cam_rays, sc, cam, a, dyn, n, stream, block, e0, e1);
  return hipErrorInvalidValue;
}

}  // namespace rtamd
