// rt_pow.hpp — `f64::powf` (material.rs:76) bit for bit as the reference's
// host computes it: glibc 2.35's pow (sysdeps/ieee754/dbl-64/e_pow.c, the ARM
// optimized-routines algorithm) in the form x86-64 selects on FMA hardware
// (the multiarch __pow_fma, where the compiler fuses each multiply that feeds
// one add into an FMA). glibc's pow is not correctly rounded (its error bound is
// 0.52 ulp: about 1 in 1300 results of x^50..x^300 differ from the correctly
// rounded value), so only its own operations reproduce its results.
//
// pow(x, y) = exp(y log x): log x = k ln2 + log c + log1p(z/c - 1) in a
// double-double (hi, lo) from a 128-entry table (1/c has few bits, so z/c - 1
// is exact) and a degree-8 polynomial; then exp of (y hi, y lo + the FMA
// residue) from a 128-entry table of 2^(k/128) and a degree-5 polynomial.
// Tables: rt_pow_tables.hpp (tools/gen_pow_tables.py). Checked against the
// host's glibc pow on random and edge inputs by tests/test_pow.py.
//
// Every input takes glibc's path, its special cases included (zero, negative,
// infinite and NaN x; zero, tiny, huge, infinite and NaN y; negative x with
// an odd integer y gives the sign), so no other pow is ever called (`lighting`
// itself passes x = reflect_dot_eye > 0, y = shininess).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_pow_tables.hpp"

namespace rtamd {

__host__ __device__ __forceinline__ uint64_t pow_bits(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double pow_dbl(uint64_t u) { return __builtin_bit_cast(double, u); }

// log_inline (e_pow.c): log(x) = hi + lo for the bits ix of a positive normal x
__host__ __device__ __forceinline__ double pow_log_inline(uint64_t ix, double* tail) {
  constexpr double Ln2hi = 0x1.62e42fefa3800p-1, Ln2lo = 0x1.ef35793c76730p-45;
  constexpr double A0 = -0x1p-1, A1 = 0x1.555555555556p-2 * -2, A2 = -0x1.0000000000006p-2 * -2,
                   A3 = 0x1.999999959554ep-3 * 4, A4 = -0x1.555555529a47ap-3 * 4,
                   A5 = 0x1.2495b9b4845e9p-3 * -8, A6 = -0x1.0002b8b263fc3p-3 * -8;
  constexpr uint64_t OFF = 0x3fe6955500000000ull;
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> 45) % 128);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = pow_dbl(iz);
  const double kd = (double)k;
  const double invc = kPowLogTab[i][0], logc = kPowLogTab[i][1], logctail = kPowLogTab[i][2];
  const double r = __builtin_fma(z, invc, -1.0);  // exact: 1/c has few bits
  const double t1 = __builtin_fma(kd, Ln2hi, logc);
  const double t2 = t1 + r;
  const double lo1 = __builtin_fma(kd, Ln2lo, logctail);
  const double lo2 = t1 - t2 + r;
  const double ar = A0 * r;
  const double ar2 = r * ar;
  const double ar3 = r * ar2;
  const double hi = t2 + ar2;
  const double lo3 = __builtin_fma(ar, r, -ar2);
  const double lo4 = t2 - hi + ar2;
  const double q = __builtin_fma(ar2, __builtin_fma(ar2, __builtin_fma(r, A6, A5), __builtin_fma(r, A4, A3)),
                                 __builtin_fma(r, A2, A1));
  const double lo = __builtin_fma(ar3, q, lo1 + lo2 + lo3 + lo4);
  const double y = hi + lo;
  *tail = hi - y + lo;
  return y;
}

constexpr uint64_t kPowSignBias = 0x800ull << 7;  // SIGN_BIAS: the result's sign through exp_inline

// exp_inline's special case (e_exp.c specialcase): the scale's exponent
// overflowed (k > 0) or the result is subnormal (k < 0)
__host__ __device__ __forceinline__ double pow_exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000ull) == 0) {
    sbits -= 1009ull << 52;
    const double scale = pow_dbl(sbits);
    return 0x1p1009 * __builtin_fma(scale, tmp, scale);
  }
  sbits += 1022ull << 52;
  const double scale = pow_dbl(sbits);
  const double st = scale * tmp;
  double y = scale + st;
  if (__builtin_fabs(y) < 1.0) {
    // round y to the subnormal grid before scaling it there (no double rounding)
    const double one = y < 0.0 ? -1.0 : 1.0;
    double lo = scale - y + st;
    const double hi = one + y;
    lo = one - hi + y + lo;
    y = (hi + lo) - one;
    if (y == 0.0) y = pow_dbl(sbits & 0x8000000000000000ull);
  }
  return 0x1p-1022 * y;
}

// exp_inline (e_pow.c): exp(x + xtail), negated when sign_bias is set
__host__ __device__ __forceinline__ double pow_exp_inline(double x, double xtail, uint64_t sign_bias) {
  constexpr double InvLn2N = 0x1.71547652b82fep0 * 128, Shift = 0x1.8p52;
  constexpr double NegLn2hiN = -0x1.62e42fefa0000p-8, NegLn2loN = -0x1.cf79abc9e3b3ap-47;
  constexpr double C2 = 0x1.ffffffffffdbdp-2, C3 = 0x1.555555555543cp-3, C4 = 0x1.55555cf172b91p-5,
                   C5 = 0x1.1111167a4d017p-7;
  auto top12 = [](double v) { return (uint32_t)(pow_bits(v) >> 52); };
  uint32_t abstop = top12(x) & 0x7ff;
  if (abstop - top12(0x1p-54) >= top12(512.0) - top12(0x1p-54)) {
    if (abstop - top12(0x1p-54) >= 0x80000000u) {  // tiny x
      const double one = 1.0 + x;
      return sign_bias ? -one : one;
    }
    if (abstop >= top12(1024.0)) {  // __math_uflow / __math_oflow
      const double r = (pow_bits(x) >> 63) ? 0x1p-767 * 0x1p-767 : 0x1p769 * 0x1p769;
      return sign_bias ? -r : r;
    }
    abstop = 0;  // large |x|: specialcase below
  }
  double kd = __builtin_fma(InvLn2N, x, Shift);
  const uint64_t ki = pow_bits(kd);
  kd -= Shift;
  double r = __builtin_fma(kd, NegLn2loN, __builtin_fma(kd, NegLn2hiN, x));
  r += xtail;
  const uint64_t idx = 2 * (ki % 128);
  const uint64_t top = (ki + sign_bias) << (52 - 7);
  const double tail = pow_dbl(kExpTab[idx]);
  const uint64_t sbits = kExpTab[idx + 1] + top;
  const double r2 = r * r;
  const double r4 = r2 * r2;
  const double tmp = __builtin_fma(r4, __builtin_fma(r, C5, C4), __builtin_fma(r2, __builtin_fma(r, C3, C2), tail + r));
  if (abstop == 0) return pow_exp_special(tmp, sbits, ki);
  const double scale = pow_dbl(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// checkint (e_pow.c): 0 = y is not an integer, 1 = an odd integer, 2 = an even one
__host__ __device__ __forceinline__ int pow_checkint(uint64_t iy) {
  const int e = (int)(iy >> 52 & 0x7ff);
  if (e < 0x3ff) return 0;
  if (e > 0x3ff + 52) return 2;
  if (iy & ((1ull << (0x3ff + 52 - e)) - 1)) return 0;
  if (iy & (1ull << (0x3ff + 52 - e))) return 1;
  return 2;
}

// pow(x, y) (glibc 2.35 __pow, FMA form)
__host__ __device__ __forceinline__ double pow_glibc(double x, double y) {
  uint64_t sign_bias = 0;
  uint64_t ix = pow_bits(x);
  const uint64_t iy = pow_bits(y);
  uint32_t topx = (uint32_t)(ix >> 52);
  const uint32_t topy = (uint32_t)(iy >> 52);
  if (topx - 0x001u >= 0x7ffu - 0x001u || (topy & 0x7ffu) - 0x3beu >= 0x43eu - 0x3beu) {
    auto zeroinfnan = [](uint64_t u) { return 2 * u - 1 >= 2 * pow_bits(__builtin_inf()) - 1; };
    if (zeroinfnan(iy)) {
      if (2 * iy == 0) return 1.0;
      if (ix == pow_bits(1.0)) return 1.0;
      if (2 * ix > 2 * pow_bits(__builtin_inf()) || 2 * iy > 2 * pow_bits(__builtin_inf())) return x + y;
      if (2 * ix == 2 * pow_bits(1.0)) return 1.0;
      if ((2 * ix < 2 * pow_bits(1.0)) == !(iy >> 63)) return 0.0;
      return y * y;
    }
    if (zeroinfnan(ix)) {
      double x2 = x * x;
      if ((ix >> 63) && pow_checkint(iy) == 1) x2 = -x2;
      return (iy >> 63) ? 1.0 / x2 : x2;
    }
    if (ix >> 63) {  // finite x < 0
      const int yint = pow_checkint(iy);
      if (yint == 0) return (x - x) / (x - x);  // __math_invalid: NaN
      if (yint == 1) sign_bias = kPowSignBias;
      ix &= 0x7fffffffffffffffull;
      topx &= 0x7ffu;
    }
    if ((topy & 0x7ffu) - 0x3beu >= 0x43eu - 0x3beu) {
      if (ix == pow_bits(1.0)) return 1.0;
      if ((topy & 0x7ffu) < 0x3beu) return ix > pow_bits(1.0) ? 1.0 + y : 1.0 - y;
      return (ix > pow_bits(1.0)) == (topy < 0x800u) ? 0x1p769 * 0x1p769 : 0x1p-767 * 0x1p-767;
    }
    if (topx == 0) {  // subnormal x: normalise, the exponent becomes negative
      ix = pow_bits(x * 0x1p52);
      ix &= 0x7fffffffffffffffull;
      ix -= 52ull << 52;
    }
  }
  double lo;
  const double hi = pow_log_inline(ix, &lo);
  const double ehi = y * hi;
  const double elo = __builtin_fma(y, lo, __builtin_fma(y, hi, -ehi));
  return pow_exp_inline(ehi, elo, sign_bias);
}

}  // namespace rtamd
