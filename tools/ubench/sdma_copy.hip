// Probe: device-to-host copy of a C3 canvas (1920x1080x3 f64 = 49.8 MB) into a
// hipHostRegister'ed host buffer, (a) with hipMemcpyAsync (ROCclr runs it as a
// blit kernel on the CUs) and (b) on the GPU's SDMA engines through
// hsa_amd_memory_async_copy_on_engine, each alone and beside a kernel that keeps
// every CU busy for ~1 ms (the render it would overlap). Prints medians of 15.
// Build: hipcc --offload-arch=gfx950 -O2 sdma_copy.hip -lhsa-runtime64 -o sdma_copy
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define HK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { const char* m_ = ""; hsa_status_string(s_, &m_); fprintf(stderr, "%s:%d hsa %d %s\n", __FILE__, __LINE__, (int)s_, m_); exit(1); } } while (0)

// one 1024-thread block per CU holding ~150 KB of LDS, like the render's LDS image
__global__ __launch_bounds__(1024) void busy(double* out, int iters) {
  extern __shared__ double lds[];
  double a = threadIdx.x * 1e-3, b = 1.0000001;
  lds[threadIdx.x] = a;
  __syncthreads();
  for (int i = 0; i < iters; ++i) a = a * b + lds[(threadIdx.x + i) & 1023] * 1e-30;
  if (a == 12345.0) out[blockIdx.x] = a;  // never true: keeps the loop
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) g_gpu = a;
  if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)1920 * 1080 * 3 * 8;
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  CK(hipSetDevice(0));
  double* src;
  CK(hipMalloc(&src, bytes));
  CK(hipMemset(src, 0x3f, bytes));
  double* dummy;
  CK(hipMalloc(&dummy, 1 << 20));
  void* host = aligned_alloc(4096, bytes);
  memset(host, 0, bytes);
  CK(hipHostRegister(host, bytes, hipHostRegisterPortable));
  void* host_dev = nullptr;
  CK(hipHostGetDevicePointer(&host_dev, host, 0));
  printf("host %p device-view %p\n", host, host_dev);
  HK(hsa_init());
  HK(hsa_iterate_agents(find_agents, nullptr));
  uint32_t pref = 0, avail = 0;
  hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &pref);
  hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &avail);
  printf("sdma engines GPU->CPU: preferred mask 0x%x, available mask 0x%x\n", pref, avail);
  hsa_signal_t sig[4];
  for (auto& s : sig) HK(hsa_signal_create(1, 0, nullptr, &s));
  hipStream_t sk, sc;
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  CK(hipFuncSetAttribute((const void*)busy, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
  CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  const int blocks = 256 * 2;

  auto sdma = [&](int parts, uint32_t mask) {
    // split into `parts` pieces over the engines in `mask` (round-robin)
    std::vector<uint32_t> eng;
    for (int b = 0; b < 16; ++b) if (mask & (1u << b)) eng.push_back(1u << b);
    if (eng.empty()) eng.push_back(1u);
    const size_t per = (bytes / parts + 4095) & ~(size_t)4095;
    for (int p = 0; p < parts; ++p) {
      const size_t off = p * per, n = std::min(per, bytes - off);
      hsa_signal_store_relaxed(sig[p], 1);
      HK(hsa_amd_memory_async_copy_on_engine((char*)host_dev + off, g_cpu, (const char*)src + off, g_gpu, n, 0, nullptr,
                                             sig[p], (hsa_amd_sdma_engine_id_t)eng[p % eng.size()], true));
    }
    for (int p = 0; p < parts; ++p)
      while (hsa_signal_wait_scacquire(sig[p], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) >= 1) {}
  };
  auto blit = [&]() {
    CK(hipMemcpyAsync(host, src, bytes, hipMemcpyDeviceToHost, sc));
    CK(hipStreamSynchronize(sc));
  };
  auto kern = [&]() { busy<<<blocks, 1024, 150 * 1024, sk>>>(dummy, iters); };
  auto med = [&](const char* name, auto fn) {
    std::vector<double> t;
    for (int r = 0; r < 17; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now_ms();
      fn();
      CK(hipDeviceSynchronize());
      t.push_back(now_ms() - t0);
    }
    std::sort(t.begin() + 2, t.end());
    const double m = t[2 + 7];
    printf("%-44s %8.3f ms  (%.1f GB/s for the canvas)\n", name, m, bytes / m / 1e6);
  };
  med("kernel alone", [&]() { kern(); });
  med("blit hipMemcpyAsync alone", [&]() { blit(); });
  med("sdma engine0 alone", [&]() { sdma(1, pref ? (pref & -pref) : 1u); });
  med("sdma 2 parts over available", [&]() { sdma(2, avail ? avail : 3u); });
  med("sdma 4 parts over available", [&]() { sdma(4, avail ? avail : 15u); });
  med("kernel + blit", [&]() { kern(); blit(); });
  med("kernel + sdma 1", [&]() { kern(); sdma(1, pref ? (pref & -pref) : 1u); });
  med("kernel + sdma 2", [&]() { kern(); sdma(2, avail ? avail : 3u); });
  med("kernel + sdma 4", [&]() { kern(); sdma(4, avail ? avail : 15u); });
  // check the bytes arrived
  const unsigned char* h = (const unsigned char*)host;
  size_t bad = 0;
  for (size_t i = 0; i < bytes; i += 4099) bad += h[i] != 0x3f;
  printf("bytes check: %zu bad samples\n", bad);
  CK(hipHostUnregister(host));
  return bad ? 1 : 0;
}
