// rt_kernels.hip — batch kernels of the C-ABI (include/rt_render.h) that are
// not part of the frame pipeline: rt_hit_batch (World::intersect + hit +
// prepare_computations + schlick for explicit rays) and rt_is_shadowed_batch
// (World::is_shadowed, world.rs:95-105). One lane per ray over the generic
// trace of rt_device.hpp (scalar, wave-uniform record loads). Frames go
// through the wavefront pipeline (rt_wavefront.hip).
//
// Compiled with -ffp-contract=off; also pins `fp contract(off)`.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rt_device.hpp"
#include "rt_kernels.hpp"

#pragma clang fp contract(off)

namespace rtamd {

// rt_hit_batch: 24 doubles per ray (layout in include/rt_render.h).
__global__ __launch_bounds__(256) void hit_kernel(DevScene sc, const double* rays, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3 o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
  const V3 d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
  Hit h;
  unsigned nd = 0;
  trace<false>(sc, o, d, h, nd);
  double* r = out + (size_t)i * 24;
  for (int k = 0; k < 24; ++k) r[k] = 0.0;
  r[0] = -1.0;
  if (h.key < 0) return;
  const Comps c = prepare(sc, o, d, h);
  r[0] = c.obj; r[1] = h.t;
  r[2] = c.point.x; r[3] = c.point.y; r[4] = c.point.z;
  r[5] = c.over.x; r[6] = c.over.y; r[7] = c.over.z;
  r[8] = c.under.x; r[9] = c.under.y; r[10] = c.under.z;
  r[11] = c.eyev.x; r[12] = c.eyev.y; r[13] = c.eyev.z;
  r[14] = c.normal.x; r[15] = c.normal.y; r[16] = c.normal.z;
  r[17] = c.inside ? 1.0 : 0.0;
  const V3 rv = vreflect(d, c.normal);  // intersection.rs:101
  r[18] = rv.x; r[19] = rv.y; r[20] = rv.z;
  r[21] = c.n1; r[22] = c.n2;
  r[23] = schlick(c.eyev, c.normal, c.n1, c.n2);
}

// rt_is_shadowed_batch: World::is_shadowed for each point against one light.
__global__ __launch_bounds__(256) void shadow_kernel(DevScene sc, const double* pts, int n, int light,
                                                     uint8_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const V3 p = v3(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
  const LightRec L = sc.lights[light];
  const V3 v = vsub(v3(L.pos[0], L.pos[1], L.pos[2]), p);
  const double distance = sqrt(v.x * v.x + v.y * v.y + v.z * v.z);  // magnitude (vector.rs:21-23)
  const V3 d = vnormalize(v);
  Hit h;
  unsigned nd = 0;
  trace<true>(sc, p, d, h, nd);
  out[i] = (h.key >= 0 && h.t < distance) ? 1 : 0;
}

hipError_t launch_hit(const DevScene& sc, const double* d_rays, int n, double* d_out, hipStream_t s) {
  hipLaunchKernelGGL(hit_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sc, d_rays, n, d_out);
  return hipGetLastError();
}

hipError_t launch_shadow(const DevScene& sc, const double* d_pts, int n, int light, uint8_t* d_out,
                         hipStream_t s) {
  hipLaunchKernelGGL(shadow_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sc, d_pts, n, light, d_out);
  return hipGetLastError();
}

// Development/test hook: the specular term's pow (rt_pow.hpp) for a batch on the
// device (tests/test_gpu_pow.py compares it with the host's glibc pow).
__global__ void pow_batch(const double* x, const double* y, int n, double* out) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) out[i] = spec_pow(x[i], y[i]);
}
hipError_t launch_pow(const double* d_x, const double* d_y, int n, double* d_out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(pow_batch, dim3((n + 255) / 256), dim3(256), 0, s, d_x, d_y, n, d_out);
  return hipGetLastError();
}

}  // namespace rtamd
