// Derived from the GNU C Library 2.35 (sysdeps/ieee754/dbl-64/e_exp.c, e_log.c,
// e_pow.c and their data files), which take these algorithms from Arm's
// optimized-routines:
//   Copyright (C) 2018-2022 Free Software Foundation, Inc.
//   Copyright (c) 2018, Arm Limited.
// The GNU C Library is free software; you can redistribute it and/or modify it
// under the terms of the GNU Lesser General Public License as published by the
// Free Software Foundation; either version 2.1 of the License, or (at your
// option) any later version.  It is distributed WITHOUT ANY WARRANTY; see the
// GNU Lesser General Public License (LGPL-2.1-or-later) for details.
//
// hb_glibc_math.hpp -- glibc 2.35's exp, log and pow, bit for bit, on the
// host and on gfx950.
//
// The reference sampler's chain states pass through glibc libm: the jump
// scale pow(10, -6 + 6 alpha) (mcmc_wrapper2.c:391), the Marsaglia polar
// Gaussian's log (:966), the priors log(gaussian()) = log(c exp(-pow(d, 2)/2))
// (:761, :1175-1178), the Hastings ratio exp(...) (:492) and the tempering
// test exp(dlogL H) (:810).  glibc's results are not correctly rounded (about
// 1 in 1000 arguments differs from the correctly rounded value), so a device
// sampler that is to reproduce the reference's chains exactly must run
// glibc's own algorithms: the table-driven exp/log/pow of
// sysdeps/ieee754/dbl-64 (ARM optimized-routines), with the tables of the
// system libm (hb_glibc_tables.inc, scripts/gen_glibc_tables.py) and the
// operation order and FMA contractions of the x86-64 FMA build that glibc's
// ifunc selects on every FMA-capable host (__exp_fma / __log_fma / __pow_fma,
// read from the libm.so.6 disassembly).  Every fma() below is one
// vfmadd/vfmsub of that build; every other operation is a plain IEEE op (the
// build compiles with -ffp-contract=off, so nothing else fuses).
//
// tests/test_glibc_math.py checks these functions against the host libm on
// millions of arguments (CPU) and the device build against the host (GPU).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HBG_FN __host__ __device__ inline
#define HBG_TABLE static __constant__ const
#else
#define HBG_FN static inline
#define HBG_TABLE static const
#endif

namespace hbglibc {

#include "hb_glibc_tables.inc"

HBG_TABLE uint64_t kExpHead[14] = HBG_EXP_HEAD;
HBG_TABLE uint64_t kExpTab[256] = HBG_EXP_TAB;
HBG_TABLE uint64_t kLogHead[18] = HBG_LOG_HEAD;
HBG_TABLE uint64_t kLogTab[256] = HBG_LOG_TAB;
HBG_TABLE uint64_t kPowHead[9] = HBG_POW_HEAD;
HBG_TABLE uint64_t kPowTab[512] = HBG_POW_TAB;

// the three data tables, by pointer: the defaults live in constant memory;
// a kernel that calls these functions on every lane may stage them in LDS
// (8 KiB) to take the divergent table loads off the L2 round trip
struct Tabs {
  const uint64_t* exp;  // 256
  const uint64_t* log;  // 256
  const uint64_t* pow;  // 512
};
constexpr int kTabWords = 256 + 256 + 512;

HBG_FN double asdouble(uint64_t u) { return __builtin_bit_cast(double, u); }
HBG_FN uint64_t asuint64(double d) { return __builtin_bit_cast(uint64_t, d); }
HBG_FN double ld(const uint64_t* t, int i) { return asdouble(t[i]); }

// __exp_data.{invln2N, shift, negln2hiN, negln2loN, poly[0..3]}
#define HBG_INVLN2N ld(kExpHead, 0)
#define HBG_SHIFT ld(kExpHead, 1)
#define HBG_NEGLN2HIN ld(kExpHead, 2)
#define HBG_NEGLN2LON ld(kExpHead, 3)
#define HBG_C2 ld(kExpHead, 4)
#define HBG_C3 ld(kExpHead, 5)
#define HBG_C4 ld(kExpHead, 6)
#define HBG_C5 ld(kExpHead, 7)

// __math_oflow / __math_uflow: +-0x1p769^2 = +-inf, +-0x1p-767^2 = +-0
HBG_FN double oflow(uint32_t sign) { return (sign ? -0x1p769 : 0x1p769) * 0x1p769; }
HBG_FN double uflow(uint32_t sign) { return (sign ? -0x1p-767 : 0x1p-767) * 0x1p-767; }

// ---------------------------------------------------------------------------
// exp (e_exp.c): exp(x) = 2^(k/128) exp(r), |r| <= ln2/256
// ---------------------------------------------------------------------------
HBG_FN double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000u) == 0) {  // k > 0: the scale's exponent overflowed by <= 460
    sbits -= 1009ull << 52;
    const double scale = asdouble(sbits);
    return 0x1p1009 * __builtin_fma(scale, tmp, scale);
  }
  sbits += 1022ull << 52;  // k < 0: round once before scaling into the subnormals
  const double scale = asdouble(sbits);
  const double st = scale * tmp;
  double y = scale + st;
  if (y < 1.0) {
    double lo = (scale - y) + st;
    const double hi = 1.0 + y;
    lo = ((1.0 - hi) + y) + lo;
    y = (hi + lo) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return 0x1p-1022 * y;
}

HBG_FN double exp(double x, const Tabs& T) {
  const uint64_t ix = asuint64(x);
  uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x3fu) {  // |x| < 2^-54, |x| >= 512, inf, nan
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;
    if (abstop >= 0x409) {  // |x| >= 1024
      if (ix == 0xfff0000000000000ull) return 0.0;
      if (abstop >= 0x7ff) return 1.0 + x;
      return (ix >> 63) ? uflow(0) : oflow(0);
    }
    abstop = 0;  // large |x|: special-cased below
  }
  const double z = __builtin_fma(x, HBG_INVLN2N, HBG_SHIFT);
  const uint64_t ki = asuint64(z);
  const double kd = z - HBG_SHIFT;
  double r = __builtin_fma(kd, HBG_NEGLN2HIN, x);
  r = __builtin_fma(kd, HBG_NEGLN2LON, r);
  const int idx = 2 * (int)(ki % 128);
  const uint64_t top = ki << 45;
  const double tail = asdouble(T.exp[idx]);
  const uint64_t sbits = T.exp[idx + 1] + top;
  const double r2 = r * r;
  const double p23 = __builtin_fma(r, HBG_C3, HBG_C2);
  const double p45 = __builtin_fma(r, HBG_C5, HBG_C4);
  const double tmp = __builtin_fma(p45, r2 * r2, __builtin_fma(p23, r2, r + tail));
  if (abstop == 0) return exp_special(tmp, sbits, ki);
  const double scale = asdouble(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// ---------------------------------------------------------------------------
// log (e_log.c): log(x) = k ln2 + log(c) + log1p(z/c - 1)
// ---------------------------------------------------------------------------
HBG_FN double log(double x, const Tabs& T) {
  uint64_t ix = asuint64(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (ix - 0x3fee000000000000ull < 0x3090000000000ull) {  // x in [1 - 2^-4, 1 + 0x1.09p-4)
    if (ix == 0x3ff0000000000000ull) return 0.0;
    const double r = x - 1.0;
    // poly1 B[0..10] = __log_data.poly1 (kLogHead[7..17])
    const double B0 = ld(kLogHead, 7), B1 = ld(kLogHead, 8), B2 = ld(kLogHead, 9), B3 = ld(kLogHead, 10),
                 B4 = ld(kLogHead, 11), B5 = ld(kLogHead, 12), B6 = ld(kLogHead, 13), B7 = ld(kLogHead, 14),
                 B8 = ld(kLogHead, 15), B9 = ld(kLogHead, 16), B10 = ld(kLogHead, 17);
    double t2 = __builtin_fma(r, B2, B1);
    double t3 = __builtin_fma(r, B5, B4);
    const double r2 = r * r;
    const double t5 = __builtin_fma(r, B8, B7);
    t2 = __builtin_fma(r2, B3, t2);
    t3 = __builtin_fma(r2, B6, t3);
    const double r3 = r * r2;
    double p = __builtin_fma(r2, B9, t5);
    p = __builtin_fma(r3, B10, p);
    p = __builtin_fma(p, r3, t3);
    p = __builtin_fma(p, r3, t2);
    // rhi = r + r 2^27 - r 2^27 (both products exact)
    const double rhi = __builtin_fma(-0x1p27, r, __builtin_fma(r, 0x1p27, r));
    const double rhi2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = __builtin_fma(rhi2, B0, r);
    double lo = __builtin_fma(rhi2, B0, r - hi);
    lo = __builtin_fma(B0 * rlo, r + rhi, lo);
    return hi + __builtin_fma(p, r3, lo);
  }
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {  // x < 2^-1022, inf, nan, <= 0
    if (ix * 2 == 0) return -1.0 / 0.0;      // __math_divzero(1)
    if (ix == 0x7ff0000000000000ull) return x;
    if ((top & 0x8000) || (top & 0x7ff0) == 0x7ff0) return (x - x) / (x - x);  // __math_invalid
    ix = asuint64(x * 0x1p52);  // subnormal: normalise
    ix -= 52ull << 52;
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) % 128);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double invc = ld(T.log, 2 * i), logc = ld(T.log, 2 * i + 1);
  const double z = asdouble(iz);
  const double kd = (double)k;
  const double Ln2hi = ld(kLogHead, 0), Ln2lo = ld(kLogHead, 1);
  const double A0 = ld(kLogHead, 2), A1 = ld(kLogHead, 3), A2 = ld(kLogHead, 4), A3 = ld(kLogHead, 5),
               A4 = ld(kLogHead, 6);
  const double r = __builtin_fma(z, invc, -1.0);
  const double w = __builtin_fma(kd, Ln2hi, logc);
  const double t5 = __builtin_fma(r, A2, A1);
  const double hi = r + w;
  const double r2 = r * r;
  double lo = (w - hi) + r;
  lo = __builtin_fma(kd, Ln2lo, lo);
  const double r3 = r * r2;
  const double t6 = __builtin_fma(r, A4, A3);
  const double lo2 = __builtin_fma(r2, A0, lo);
  const double p = __builtin_fma(t6, r2, t5);
  return __builtin_fma(r3, p, lo2) + hi;
}

// ---------------------------------------------------------------------------
// pow (e_pow.c): exp(y log x) with a double-double log
// ---------------------------------------------------------------------------
HBG_FN double pow_log_inline(uint64_t ix, double* tail, const Tabs& T) {
  const uint64_t tmp = ix - 0x3fe6955500000000ull;
  const int i = (int)((tmp >> 45) % 128);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = asdouble(iz);
  const double kd = (double)k;
  const double invc = ld(T.pow, 4 * i), logc = ld(T.pow, 4 * i + 2), logctail = ld(T.pow, 4 * i + 3);
  const double Ln2hi = ld(kPowHead, 0), Ln2lo = ld(kPowHead, 1);
  const double A0 = ld(kPowHead, 2), A1 = ld(kPowHead, 3), A2 = ld(kPowHead, 4), A3 = ld(kPowHead, 5),
               A4 = ld(kPowHead, 6), A5 = ld(kPowHead, 7), A6 = ld(kPowHead, 8);
  const double t1 = __builtin_fma(kd, Ln2hi, logc);
  const double r = __builtin_fma(z, invc, -1.0);
  const double ar = r * A0;
  const double lo1 = __builtin_fma(kd, Ln2lo, logctail);
  const double q12 = __builtin_fma(r, A2, A1);
  const double q34 = __builtin_fma(r, A4, A3);
  const double t2 = r + t1;
  const double ar2 = r * ar;
  const double lo2 = (t1 - t2) + r;
  const double ar3 = r * ar2;
  const double lo3 = __builtin_fma(ar, r, -ar2);
  const double q56 = __builtin_fma(r, A6, A5);
  const double hi = t2 + ar2;
  const double lo4 = (t2 - hi) + ar2;
  const double q = __builtin_fma(ar2, __builtin_fma(q56, ar2, q34), q12);
  const double lo = __builtin_fma(ar3, q, ((lo1 + lo2) + lo3) + lo4);
  const double y = hi + lo;
  *tail = (hi - y) + lo;
  return y;
}

HBG_FN double pow_exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  if ((ki & 0x80000000u) == 0) {
    sbits -= 1009ull << 52;
    const double scale = asdouble(sbits);
    return 0x1p1009 * __builtin_fma(scale, tmp, scale);
  }
  sbits += 1022ull << 52;
  const double scale = asdouble(sbits);
  const double st = scale * tmp;
  double y = scale + st;
  if (__builtin_fabs(y) < 1.0) {
    const double one = (y < 0.0) ? -1.0 : 1.0;
    double lo = (scale - y) + st;
    const double hi = one + y;
    lo = ((one - hi) + y) + lo;
    y = (hi + lo) - one;
    if (y == 0.0) y = asdouble(sbits & 0x8000000000000000ull);
  }
  return 0x1p-1022 * y;
}

HBG_FN double pow_exp_inline(double x, double xtail, uint32_t sign_bias, const Tabs& T) {
  const uint64_t ix = asuint64(x);
  uint32_t abstop = (uint32_t)(ix >> 52) & 0x7ff;
  if (abstop - 0x3c9u >= 0x3fu) {
    if ((int32_t)(abstop - 0x3c9u) < 0) {
      const double one = 1.0 + x;
      return sign_bias ? -one : one;
    }
    if (abstop >= 0x409) return (ix >> 63) ? uflow(sign_bias) : oflow(sign_bias);
    abstop = 0;
  }
  const double z = __builtin_fma(x, HBG_INVLN2N, HBG_SHIFT);
  const uint64_t ki = asuint64(z);
  const double kd = z - HBG_SHIFT;
  double r = __builtin_fma(kd, HBG_NEGLN2HIN, x);
  r = __builtin_fma(kd, HBG_NEGLN2LON, r);
  r = xtail + r;
  const int idx = 2 * (int)(ki % 128);
  const uint64_t top = (ki + sign_bias) << 45;
  const double tail = asdouble(T.exp[idx]);
  const uint64_t sbits = T.exp[idx + 1] + top;
  const double r2 = r * r;
  const double p23 = __builtin_fma(r, HBG_C3, HBG_C2);
  const double p45 = __builtin_fma(r, HBG_C5, HBG_C4);
  const double tmp = __builtin_fma(p45, r2 * r2, __builtin_fma(p23, r2, r + tail));
  if (abstop == 0) return pow_exp_special(tmp, sbits, ki);
  const double scale = asdouble(sbits);
  return __builtin_fma(scale, tmp, scale);
}

// 0: not an integer, 1: odd integer, 2: even integer
HBG_FN int checkint(uint64_t iy) {
  const int e = (int)(iy >> 52 & 0x7ff);
  if (e < 0x3ff) return 0;
  if (e > 0x3ff + 52) return 2;
  if (iy & ((1ull << (0x3ff + 52 - e)) - 1)) return 0;
  if (iy & (1ull << (0x3ff + 52 - e))) return 1;
  return 2;
}

HBG_FN bool zeroinfnan(uint64_t i) { return 2 * i - 1 >= 2 * 0x7ff0000000000000ull - 1; }

HBG_FN double pow(double x, double y, const Tabs& T) {
  uint32_t sign_bias = 0;
  uint64_t ix = asuint64(x);
  const uint64_t iy = asuint64(y);
  uint32_t topx = (uint32_t)(ix >> 52);
  const uint32_t topy = (uint32_t)(iy >> 52);
  if (topx - 0x001u >= 0x7ffu - 0x001u || (topy & 0x7ff) - 0x3beu >= 0x43eu - 0x3beu) {
    if (zeroinfnan(iy)) {
      if (2 * iy == 0) return 1.0;
      if (ix == 0x3ff0000000000000ull) return 1.0;
      if (2 * ix > 2 * 0x7ff0000000000000ull || 2 * iy > 2 * 0x7ff0000000000000ull) return x + y;
      if (2 * ix == 2 * 0x3ff0000000000000ull) return 1.0;
      if ((2 * ix < 2 * 0x3ff0000000000000ull) == !(iy >> 63)) return 0.0;
      return y * y;
    }
    if (zeroinfnan(ix)) {
      double x2 = x * x;
      if ((ix >> 63) && checkint(iy) == 1) x2 = -x2;
      return (iy >> 63) ? 1.0 / x2 : x2;
    }
    if (ix >> 63) {  // finite x < 0
      const int yint = checkint(iy);
      if (yint == 0) return (x - x) / (x - x);
      if (yint == 1) sign_bias = 0x800 << 7;
      ix &= 0x7fffffffffffffffull;
      topx &= 0x7ff;
    }
    if ((topy & 0x7ff) - 0x3beu >= 0x43eu - 0x3beu) {
      if (ix == 0x3ff0000000000000ull) return 1.0;
      if ((topy & 0x7ff) < 0x3be) return ix > 0x3ff0000000000000ull ? 1.0 + y : 1.0 - y;
      return (ix > 0x3ff0000000000000ull) == (topy < 0x800) ? oflow(0) : uflow(0);
    }
    if (topx == 0) {  // subnormal x
      ix = asuint64(x * 0x1p52);
      ix &= 0x7fffffffffffffffull;
      ix -= 52ull << 52;
    }
  }
  double lo;
  const double hi = pow_log_inline(ix, &lo, T);
  const double ehi = y * hi;
  const double elo = __builtin_fma(y, lo, __builtin_fma(y, hi, -ehi));
  return pow_exp_inline(ehi, elo, sign_bias, T);
}

// the same functions with the constant-memory tables
HBG_FN Tabs const_tabs() { return Tabs{kExpTab, kLogTab, kPowTab}; }
HBG_FN double exp(double x) { return exp(x, const_tabs()); }
HBG_FN double log(double x) { return log(x, const_tabs()); }
HBG_FN double pow(double x, double y) { return pow(x, y, const_tabs()); }

}  // namespace hbglibc
