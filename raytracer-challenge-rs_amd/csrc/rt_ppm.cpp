// rt_ppm.cpp — output side of the path (image/ppm.rs): the bit-exact P3 writer.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/rt_render.h"

namespace {

// image/ppm.rs:73-75: `(value * 255.0).round() as u8` — C round() is half away
// from zero like f64::round; the `as u8` cast saturates and maps NaN to 0.
inline unsigned scale_color_component(double v) {
  const double s = std::round(v * 255.0);
  if (!(s > 0.0)) return 0;
  if (s >= 255.0) return 255;
  return (unsigned)s;
}

inline int utoa3(unsigned v, char* out) {  // v <= 255
  if (v >= 100) { out[0] = char('0' + v / 100); out[1] = char('0' + (v / 10) % 10); out[2] = char('0' + v % 10); return 3; }
  if (v >= 10) { out[0] = char('0' + v / 10); out[1] = char('0' + v % 10); return 2; }
  out[0] = char('0' + v);
  return 1;
}

}  // namespace

extern "C" {

int rt_quantize_u8(const double* values, size_t n, uint8_t* out) {
  if (n && (!values || !out)) return RT_ERR_INVALID_ARGUMENT;
  for (size_t i = 0; i < n; ++i) out[i] = (uint8_t)scale_color_component(values[i]);
  return RT_OK;
}

// image/ppm.rs:24-63. Tokens are appended to the current line; before each
// token, if line.len() + token.len() > 70 the line is flushed with its
// trailing spaces trimmed (`trim_end`). Each canvas row ends the line.
int rt_canvas_to_ppm(const double* rgb, uint32_t width, uint32_t height, char* out, size_t cap,
                     size_t* out_len) {
  if (!out_len || (width && height && !rgb)) return RT_ERR_INVALID_ARGUMENT;
  size_t len = 0;
  auto emit = [&](const char* s, size_t n) {
    if (out && len + n <= cap) std::memcpy(out + len, s, n);
    len += n;
  };
  char hdr[64];
  int hn = std::snprintf(hdr, sizeof hdr, "P3\n%u %u\n255\n", width, height);
  emit(hdr, (size_t)hn);
  char line[96];
  for (uint32_t j = 0; j < height; ++j) {
    size_t ll = 0;
    for (uint32_t i = 0; i < width; ++i) {
      const double* px = rgb + ((size_t)j * width + i) * 3;
      for (int idx = 0; idx < 3; ++idx) {
        char tok[4];
        const int tn = utoa3(scale_color_component(px[idx]), tok);
        if (ll + (size_t)tn > 70) {
          size_t tl = ll;
          while (tl > 0 && line[tl - 1] == ' ') --tl;
          emit(line, tl);
          emit("\n", 1);
          ll = 0;
        }
        std::memcpy(line + ll, tok, (size_t)tn);
        ll += (size_t)tn;
        if (idx < 2) line[ll++] = ' ';
      }
      if (i + 1 < width) line[ll++] = ' ';
    }
    emit(line, ll);
    emit("\n", 1);
  }
  *out_len = len;
  if (out && len > cap) return RT_ERR_BUFFER_TOO_SMALL;
  return RT_OK;
}

}  // extern "C"
