// f64 VALU microbenchmark (dev tool): throughput of non-fused v_mul_f64 /
// v_add_f64 vs the number of independent chains per wave and waves per SIMD.
// Pins the peak used by the roofline (DESIGN.md "Roofline").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#pragma clang fp contract(off)

template <int CHAINS>
__global__ void chains(double* out, int iters, double a, double b) {
  double x[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      x[c] = x[c] * a;  // v_mul_f64
      x[c] = x[c] + b;  // v_add_f64
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
void run(int waves_per_simd, int n_cu) {
  const int block = 256;  // 4 waves: one per SIMD
  const int blocks = n_cu * waves_per_simd;
  const int iters = 4096;
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * block);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(chains<CHAINS>, dim3(blocks), dim3(block), 0, 0, out, iters, 0.999999, 1e-9);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(chains<CHAINS>, dim3(blocks), dim3(block), 0, 0, out, iters, 0.999999, 1e-9);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double ops = 5.0 * blocks * block * (double)iters * CHAINS * 2;
  printf("chains=%2d waves/SIMD=%d  %.2f Tops/s\n", CHAINS, waves_per_simd, ops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  int n_cu = 0;
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", n_cu);
  for (int w : {1, 2, 3, 4, 8}) {
    run<1>(w, n_cu); run<2>(w, n_cu); run<4>(w, n_cu); run<8>(w, n_cu);
  }
  return 0;
}
