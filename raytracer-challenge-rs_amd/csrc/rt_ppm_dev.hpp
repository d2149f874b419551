// rt_ppm_dev.hpp — canvas_to_ppm on the device (rt_ppm_dev.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rtamd {

// A row's text is staged in LDS (<= 12 bytes per pixel).
constexpr uint32_t kPpmMaxWidth = 12288;

struct PpmHeader {  // "P3\n{w} {h}\n255\n" (image/ppm.rs:53-63)
  char s[48];
  unsigned n;
};

size_t ppm_device_max_width();

// Encodes the H x W x 3 f64 canvas at d_rgb into d_out (cap bytes): the header,
// then every row's text. d_row_len: H words; d_row_off: H + 1 words, of which
// d_row_off[H] receives the body's length (the text is hdr.n + d_row_off[H]
// bytes). Rows that do not fit in cap are not written. d_out == nullptr: the
// lengths only. Stream-ordered; nothing is synchronised.
hipError_t ppm_encode_device(const double* d_rgb, uint32_t W, uint32_t H, char* d_out, unsigned long long cap,
                             unsigned* d_row_len, unsigned long long* d_row_off, const PpmHeader& hdr,
                             hipStream_t stream);

}  // namespace rtamd
