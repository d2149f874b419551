// rt_ppm.cpp — output side of the path (image/ppm.rs): the bit-exact P3 writer.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>
#include <atomic>

#include "../../include/rt_render.h"

namespace {

// image/ppm.rs:73-75: `(value * 255.0).round() as u8` — C round() is half away
// from zero like f64::round; the `as u8` cast saturates and maps NaN to 0.
// round(s) for 0 < s < 254.5 without a libm call: the truncating conversion
// is exact there, and so is s - trunc(s), so `frac >= 0.5` is round's
// half-away-from-zero rule exactly.
inline unsigned scale_color_component(double v) {
  const double s = v * 255.0;
  if (!(s >= 0.5)) return 0;  // also NaN (as u8: 0) and everything that rounds to <= 0
  if (s >= 254.5) return 255;
  const unsigned i = (unsigned)s;
  return i + (s - (double)i >= 0.5 ? 1u : 0u);
}

// "0".."255" as up to three digit bytes, with the token length in byte 3
struct DigitTable {
  uint32_t t[256];
  DigitTable() {
    for (unsigned v = 0; v < 256; ++v) {
      char b[4] = {0, 0, 0, 0};
      const int n = v >= 100 ? 3 : v >= 10 ? 2 : 1;
      for (int k = n - 1, x = (int)v; k >= 0; --k, x /= 10) b[k] = char('0' + x % 10);
      b[3] = (char)n;
      std::memcpy(&t[v], b, 4);
    }
  }
};
const DigitTable kDigits;

inline unsigned tok_len(unsigned q) { return kDigits.t[q] >> 24; }

}  // namespace

extern "C" {

int rtamd_fail(int code, const char* msg) noexcept;  // rt_api.cpp

int rt_quantize_u8(const double* values, size_t n, uint8_t* out) {
  if (n && (!values || !out)) return rtamd_fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  for (size_t i = 0; i < n; ++i) out[i] = (uint8_t)scale_color_component(values[i]);
  return RT_OK;
}

// image/ppm.rs:24-63. Tokens are appended to the current line; before each
// token, if line.len() + token.len() > 70 the line is flushed with its
// trailing spaces trimmed (`trim_end`), and each canvas row ends the line.
// Every token but the row's last is followed by exactly one space, and a flush
// turns that one space into '\n', so a row's text is its tokens joined by one
// separator byte each plus the final '\n' (its length does not depend on the
// breaks), and the breaks are found afterwards: with the line starting at byte
// ls, the last space at or before byte ls + 70 becomes '\n' whenever the row's
// last token ends beyond ls + 70 (rt_ppm_dev.hip uses the same two facts).
// Rows are encoded in parallel.
}  // extern "C"

namespace {

size_t ppm_row_len(const double* row, uint32_t w) {
  if (w == 0) return 1;
  size_t n = 0;
  for (size_t k = 0; k < (size_t)3 * w; ++k) n += tok_len(scale_color_component(row[k])) + 1;
  return n;
}

void ppm_row_write(const double* row, uint32_t w, char* out) {
  char* p = out;
  const size_t n = (size_t)3 * w;
  for (size_t k = 0; k + 1 < n; ++k) {
    // 4-byte store: the digits, then the separator over the length byte (the
    // row's bytes are exactly its tokens + separators, so this stays inside it)
    const uint32_t d = kDigits.t[scale_color_component(row[k])];
    const unsigned len = d >> 24;
    std::memcpy(p, &d, 4);
    p[len] = ' ';
    p += len + 1;
  }
  if (n) {  // the last token: byte by byte (the store above could pass the row's end)
    const uint32_t d = kDigits.t[scale_color_component(row[n - 1])];
    const unsigned len = d >> 24;
    for (unsigned k = 0; k < len; ++k) p[k] = (char)(d >> (8 * k));
    p += len;
  }
  *p++ = '\n';
  const size_t len = (size_t)(p - out);
  size_t ls = 0;
  while (ls + 70 < len - 1) {
    size_t q = ls + 70;
    while (out[q] != ' ') --q;
    out[q] = '\n';
    ls = q + 1;
  }
}

// The rows in kBlocks contiguous blocks, encoded by the calling thread and up
// to kBlocks - 1 helpers started once: every participant takes blocks from a
// counter, first measuring them (each row's text length), then, once every
// block is measured, writing them at their offsets (header + the lengths of the
// rows before). Any number of participants (one, if no thread can start)
// finishes every block.
constexpr unsigned kBlocks = 16;

struct PpmJob {
  const double* rgb = nullptr;
  uint32_t width = 0, height = 0;
  char* out = nullptr;  // nullptr: measure only
  size_t hn = 0, row_doubles = 0;
  uint32_t* row_len = nullptr;  // per row, filled by the measuring pass
  size_t block_len[kBlocks] = {};
  std::atomic<unsigned> next1{0}, done1{0}, next2{0};
  uint32_t r0(unsigned b) const { return (uint32_t)(((uint64_t)height * b) / kBlocks); }
  void run() {
    for (unsigned b; (b = next1.fetch_add(1)) < kBlocks;) {
      size_t n = 0;
      for (uint32_t j = r0(b); j < r0(b + 1); ++j) {
        row_len[j] = (uint32_t)ppm_row_len(rgb + j * row_doubles, width);
        n += row_len[j];
      }
      block_len[b] = n;
      done1.fetch_add(1, std::memory_order_release);
    }
    if (!out) return;
    while (done1.load(std::memory_order_acquire) < kBlocks) std::this_thread::yield();
    for (unsigned b; (b = next2.fetch_add(1)) < kBlocks;) {
      size_t off = hn;
      for (unsigned k = 0; k < b; ++k) off += block_len[k];
      for (uint32_t j = r0(b); j < r0(b + 1); ++j) {
        ppm_row_write(rgb + j * row_doubles, width, out + off);
        off += row_len[j];
      }
    }
  }
  // run() on the calling thread and up to `t` - 1 helpers
  void run_on(unsigned t) {
    std::vector<std::thread> pool;
    try {  // nothing may throw across the C ABI: blocks whose thread cannot start run here
      for (unsigned k = 1; k < t; ++k) pool.emplace_back([this] { run(); });
    } catch (...) {
    }
    run();
    for (std::thread& th : pool) th.join();
  }
};

}  // namespace

extern "C" {

int rt_canvas_to_ppm(const double* rgb, uint32_t width, uint32_t height, char* out, size_t cap,
                     size_t* out_len) {
  if (!out_len || (width && height && !rgb)) return rtamd_fail(RT_ERR_INVALID_ARGUMENT, "null pointer");
  char hdr[64];
  const size_t hn = (size_t)std::snprintf(hdr, sizeof hdr, "P3\n%u %u\n255\n", width, height);
  std::vector<uint32_t> row_len;
  try {
    row_len.assign((size_t)height + 1, 0);
  } catch (...) {  // nothing may throw across the C ABI (as guarded() in rt_api.cpp)
    return rtamd_fail(RT_ERR_HOST, "out of memory (PPM row lengths)");
  }
  const size_t row_doubles = (size_t)width * 3;
  unsigned t = std::thread::hardware_concurrency();
  t = std::max(1u, std::min(t, kBlocks));
  if (row_doubles * height < ((size_t)1 << 18) || height < 2 * kBlocks) t = 1;
  auto init = [&](PpmJob& j, char* dst) {
    j.rgb = rgb; j.width = width; j.height = height; j.out = dst; j.hn = hn;
    j.row_doubles = row_doubles; j.row_len = row_len.data();
  };
  // one pass (measure, then write) when the buffer holds the bound (12 bytes per
  // pixel, a newline per row, the header); otherwise measure, check, then write
  const size_t bound = hn + (size_t)12 * width * height + height;
  const bool one_pass = out && cap >= bound;
  size_t len = hn;
  {
    PpmJob j;
    init(j, one_pass ? out : nullptr);
    if (one_pass) std::memcpy(out, hdr, hn);
    j.run_on(t);
    for (unsigned b = 0; b < kBlocks; ++b) len += j.block_len[b];
  }
  *out_len = len;
  if (!out || one_pass) return RT_OK;
  if (len > cap) return rtamd_fail(RT_ERR_BUFFER_TOO_SMALL, "PPM buffer too small");
  std::memcpy(out, hdr, hn);
  PpmJob j;
  init(j, out);
  j.run_on(t);
  return RT_OK;
}

}  // extern "C"
