// rt_ppm_dev.hip — canvas_to_ppm (image/ppm.rs:24-75) on the device.
//
// The reference builds the P3 text row by row: every component becomes the
// decimal token of `(v * 255.0).round() as u8` (ppm.rs:73-75), tokens are
// joined by one space, and before a token that would take the line past 70
// characters the line is flushed with its trailing space trimmed and a newline
// (ppm.rs:29-46); each canvas row ends its last line with a newline (:47-48).
//
// Two facts make this parallel:
//  - Every token except the row's last is followed by exactly one space, and a
//    flush replaces that one trailing space with '\n'. So the byte position of
//    every token does not depend on where the lines break: a row's text is its
//    tokens joined by one separator byte each, plus the final '\n', and its
//    length is the sum over its tokens of (digits + 1).
//  - The greedy break rule only picks WHICH separators become '\n'. With the
//    line starting at byte ls, the first token that no longer fits is the first
//    one ending after byte ls + 70; its separator is the last space at or
//    before byte ls + 70 (tokens are 1-3 bytes), which becomes '\n', and the
//    next line starts after it. One thread walks a row in ~len/70 such steps.
//
// Kernels: row lengths (one block per row), one exclusive scan over the rows,
// then one block per row writes its text into LDS, walks its breaks and copies
// the row to out[header + row offset]. Bytes are identical to rt_canvas_to_ppm
// (host) and to the oracle's writer; tests/test_gpu_ppm.py checks them.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_ppm_dev.hpp"

namespace rtamd {
namespace {

constexpr int kPpmBlock = 256;

// scale_color_component (ppm.rs:73-75): round() is half away from zero like
// f64::round; `as u8` saturates and maps NaN to 0.
__device__ __forceinline__ unsigned q255(double v) {
  const double s = round(v * 255.0);
  if (!(s > 0.0)) return 0u;
  if (s >= 255.0) return 255u;
  return (unsigned)s;
}
__device__ __forceinline__ unsigned n_digits(unsigned q) { return q >= 100u ? 3u : q >= 10u ? 2u : 1u; }

// The thread's contiguous range of pixels of a row of W.
__device__ __forceinline__ void pixel_range(unsigned W, unsigned& x0, unsigned& x1) {
  const unsigned c = (W + kPpmBlock - 1) / kPpmBlock;
  x0 = min(W, threadIdx.x * c);
  x1 = min(W, x0 + c);
}

// Bytes of pixels [x0, x1) of a row: each component's digits plus its separator.
__device__ __forceinline__ unsigned range_bytes(const double* row, unsigned x0, unsigned x1) {
  unsigned n = 0;
  for (unsigned k = 3 * x0; k < 3 * x1; ++k) n += n_digits(q255(row[k])) + 1u;
  return n;
}

// Block-wide exclusive scan of 256 values; *total receives the sum.
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* total) {
  __shared__ T wave_sum[kPpmBlock / 64];
  const unsigned lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  T incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T t = __shfl_up(incl, off, 64);
    if ((int)lane >= off) incl += t;
  }
  if (lane == 63) wave_sum[wave] = incl;
  __syncthreads();
  T before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kPpmBlock / 64; ++w) {
    if ((unsigned)w < wave) before += wave_sum[w];
    all += wave_sum[w];
  }
  *total = all;
  return before + incl - v;
}

__global__ __launch_bounds__(kPpmBlock) void ppm_row_len(const double* rgb, unsigned W, unsigned* row_len) {
  const unsigned j = blockIdx.x;
  unsigned x0, x1;
  pixel_range(W, x0, x1);
  const unsigned mine = range_bytes(rgb + (size_t)j * W * 3, x0, x1);
  unsigned total;
  (void)block_exclusive_scan<unsigned>(mine, &total);
  if (threadIdx.x == 0) row_len[j] = W ? total : 1u;  // an empty row is "\n" (ppm.rs:47-48)
}

// One block: exclusive prefix of the H row lengths; row_off[H] = the body's length.
__global__ __launch_bounds__(kPpmBlock) void ppm_scan_rows(const unsigned* row_len, unsigned H,
                                                          unsigned long long* row_off) {
  const unsigned c = (H + kPpmBlock - 1) / kPpmBlock;
  const unsigned r0 = min(H, threadIdx.x * c), r1 = min(H, r0 + c);
  unsigned long long mine = 0;
  for (unsigned r = r0; r < r1; ++r) mine += row_len[r];
  unsigned long long total;
  unsigned long long off = block_exclusive_scan<unsigned long long>(mine, &total);
  for (unsigned r = r0; r < r1; ++r) {
    row_off[r] = off;
    off += row_len[r];
  }
  if (threadIdx.x == 0) row_off[H] = total;
}

__device__ __forceinline__ unsigned put_token(char* p, unsigned q) {
  if (q >= 100u) {
    p[0] = (char)('0' + q / 100u); p[1] = (char)('0' + (q / 10u) % 10u); p[2] = (char)('0' + q % 10u);
    return 3u;
  }
  if (q >= 10u) {
    p[0] = (char)('0' + q / 10u); p[1] = (char)('0' + q % 10u);
    return 2u;
  }
  p[0] = (char)('0' + q);
  return 1u;
}

__global__ __launch_bounds__(kPpmBlock) void ppm_row_write(const double* rgb, unsigned W,
                                                          const unsigned long long* row_off, PpmHeader hdr,
                                                          char* out, unsigned long long cap) {
  extern __shared__ char text[];
  const unsigned j = blockIdx.x;
  const double* row = rgb + (size_t)j * W * 3;
  unsigned x0, x1;
  pixel_range(W, x0, x1);
  unsigned len;
  unsigned pos = block_exclusive_scan<unsigned>(range_bytes(row, x0, x1), &len);
  for (unsigned k = 3 * x0; k < 3 * x1; ++k) {
    pos += put_token(text + pos, q255(row[k]));
    text[pos++] = (k + 1 == 3 * W) ? '\n' : ' ';  // the row's last token ends it (ppm.rs:47-48)
  }
  if (W == 0) {
    len = 1;
    if (threadIdx.x == 0) text[0] = '\n';
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // greedy 70-column breaks (ppm.rs:33-37): the last token ends at len - 1
    unsigned ls = 0;
    while (ls + 70u < len - 1u) {
      unsigned q = ls + 70u;
      while (text[q] != ' ') --q;
      text[q] = '\n';
      ls = q + 1u;
    }
  }
  __syncthreads();
  const unsigned long long base = hdr.n + row_off[j];
  if (base + len <= cap)  // rows that do not fit are not written (RT_ERR_BUFFER_TOO_SMALL)
    for (unsigned k = threadIdx.x; k < len; k += kPpmBlock) out[base + k] = text[k];
  if (j == 0 && threadIdx.x < hdr.n && hdr.n <= cap) out[threadIdx.x] = hdr.s[threadIdx.x];
}

}  // namespace

size_t ppm_device_max_width() { return kPpmMaxWidth; }


hipError_t ppm_encode_device(const double* d_rgb, uint32_t W, uint32_t H, char* d_out, unsigned long long cap,
                             unsigned* d_row_len, unsigned long long* d_row_off, const PpmHeader& hdr,
                             hipStream_t stream) {
  if (W > kPpmMaxWidth || H == 0) return hipErrorInvalidValue;
  const size_t lds = (size_t)12 * W + 16;  // <= 3 digits + 1 separator per component
  hipLaunchKernelGGL(ppm_row_len, dim3(H), dim3(kPpmBlock), 0, stream, d_rgb, W, d_row_len);
  hipLaunchKernelGGL(ppm_scan_rows, dim3(1), dim3(kPpmBlock), 0, stream, d_row_len, H, d_row_off);
  if (d_out) {
    hipError_t e = hipFuncSetAttribute((const void*)ppm_row_write, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ppm_row_write, dim3(H), dim3(kPpmBlock), lds, stream, d_rgb, W,
                       (const unsigned long long*)d_row_off, hdr, d_out, cap);
  }
  return hipGetLastError();
}

}  // namespace rtamd
