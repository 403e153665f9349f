// hb_walls.hpp -- the reflecting / periodic walls of mcmc_wrapper2.c:440-467,
// bit for bit, with an exact fast-forward of long reflection runs.
//
// Hot chains (temperatures up to 1.4^49 on the 50-rung ladder) propose steps
// thousands of ranges wide, and the reference then folds the coordinate back
// one reflection at a time: v <- 2 lo - v below the range, v <- 2 hi - v above
// (each a rounded subtraction).  On a GPU lane every fold is a dependent
// step; 10^4 folds of one hot chain stall its whole wave.
//
// Fast-forward (both walls reflecting, v far outside): while |v| stays in one
// binade [2^e, 2^(e+1)) every double there is a multiple of g = 2^(e-52), and
// the exact result c - v of a fold lands in the same binade, so
//     fl(c - v) = round_g(c) - v        (translation by a grid multiple)
// unless c/g is a rounding tie (then round-half-even would depend on v: no
// fast-forward).  Two folds (2 lo then 2 hi, or the reverse) therefore move
// K = v/g by the exact integer D = round(2hi/g) - round(2lo/g); m double
// folds are K + m D.  m is capped so that every intermediate value keeps a
// margin inside the binade (and outside [lo, hi]), and so that the fold
// counter never passes the 10^8 guard of the host loop; the remaining folds
// run one by one.  tests/test_walls.py checks it against the plain loop.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HBW_FN __host__ __device__ inline
#else
#define HBW_FN static inline
#endif

namespace hbwall {

constexpr int kGuard = 100000000;  // fold bound of the host loop (hb_sampler.cpp, before hb_walls)

// floor(num / den) for exact integers 0 <= num, 1 <= den below 2^53: an
// approximate quotient corrected with exact products
HBW_FN double floor_div(double num, double den) {
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rcp(den);
  y = __builtin_fma(__builtin_fma(-den, y, 1.0), y, y);
  double q = floor(num * y);
#else
  double q = floor(num / den);
#endif
  if (q * den > num) q -= 1.0;
  if ((q + 1.0) * den <= num) q += 1.0;
  return q;
}

// Fast-forward within v's binade: returns v after 2m folds, m >= 0 (m = 0:
// not applicable, v unchanged); folds_left caps 2m.
//
// In units of g (K = |v| / g in [2^52, 2^53)): a pair of folds starting
// below the range (v < 0) takes the magnitude K -> K + rlo (first fold, the
// chain is now above hi) -> K + rlo - rhi = K - D; starting above (v > 0),
// K -> K - rhi -> K - D.  Both exact results must stay in the binade:
// K_j + c1 >= 2^52 + 1 (c1 = rlo or -rhi), K_j - D >= 2^52 + 1, and at the
// top K_0 + c1 <= 2^53 - 2.  Every magnitude of the binade exceeds
// 2 max(|lo|, |hi|), so each value lies outside [lo, hi] on its sign's side.
//
// `bottom` receives 2^eb, the lower edge of v's binade.  When no fast-forward
// is possible the caller folds one at a time; `mode` says for how long:
//   kFfTop   -- a margin at the binade top: a few folds, then try again;
//   kFfBinade -- too little room above the bottom: fold until |v| drops
//               below `bottom` (the next binade);
//   kFfNear  -- v's binade is within 2 max(|lo|, |hi|): no lower binade can
//               fast-forward either, fold to the end;
//   kFfTie   -- a rounding-tie binade: tie_double_folds.
enum { kFfDone = 0, kFfTop = 1, kFfBinade = 2, kFfNear = 3, kFfTie = 4 };
HBW_FN double ff_double_folds(double v, double lo, double hi, int folds_left, int& m_out, int& mode,
                              double& bottom) {
  // every quantity is computed unconditionally and the outcome selected at
  // the end (no early exits: on a GPU lane the tests would serialise into
  // exec-mask branches); garbage from a failed test is discarded
  const double av = fabs(v);
  const bool finite = (av < 0x1p1000) & (av > 0.0);
  int e;
  frexp(av, &e);                       // av = f 2^e, f in [0.5, 1): binade [2^(e-1), 2^e)
  const int eb = finite ? e - 1 : 0;   // av in [2^eb, 2^(eb+1))
  bottom = finite ? ldexp(1.0, eb) : 0.0;
  const double lim = fabs(lo) > fabs(hi) ? fabs(lo) : fabs(hi);
  const bool far = bottom > 2.0 * lim;
  const double scale = ldexp(1.0, 52 - eb);  // 1/g
  const double clo = 2.0 * lo * scale, chi = 2.0 * hi * scale;  // exact (power-of-2 scaling), |.| < 2^52
  const bool tie_lo = clo - floor(clo) == 0.5, tie_hi = chi - floor(chi) == 0.5;
  const bool tie = tie_lo | tie_hi;  // rounding ties: no translation
  const double rlo = rint(clo), rhi = rint(chi);
  const double D = rhi - rlo;                  // exact integer
  const double K = av * scale;                 // exact integer in [2^52, 2^53)
  const double c1 = v < 0.0 ? rlo : -rhi;
  const bool fits = (D > 0.0) & (K + (c1 > 0.0 ? c1 : 0.0) <= 0x1p53 - 2.0);
  // m pairs: K - (m-1) D + c1 >= 2^52 + 1 and K - m D >= 2^52 + 1
  const double n1 = K - 0x1p52 - 1.0, n2 = K + c1 - 0x1p52 - 1.0;
  const bool room = (n1 >= D) & (n2 >= 0.0);
  double m = floor_div(n1, D);
  const double m2 = floor_div(n2, D) + 1.0;
  if (m2 < m) m = m2;
  const double cap = (double)(folds_left / 2);
  if (m > cap) m = cap;
  const bool go = finite & far & !tie & fits & room & (m >= 1.0);
  mode = go ? kFfDone
            : !finite ? kFfTop : !far ? kFfNear : tie ? kFfTie : !fits ? kFfTop : !room ? kFfBinade : kFfTop;
  m_out = go ? (int)m : 0;
  // exact: integers below 2^53 times a power of two (g = 2^(eb-52))
  return go ? copysign((K - m * D) * ldexp(1.0, eb - 52), v) : v;
}

// Rounding-tie binade [B, 2B) far from the range (mode kFfTie): 2lo/g or
// 2hi/g is a half-integer, so that fold rounds half to even and its result
// depends on the parity of K.  The tie fold's result is always even, so after
// two plain folds the parity entering every later fold is fixed and each pair
// of folds again moves the magnitude by constants (first fold c1, the pair
// -D), which the next plain pair measures.  The remaining pairs that keep
// every value inside the binade (the margins of ff_double_folds) are then
// taken at once.  Returns v after the folds made; guard counts them.  A fold
// that leaves the binade ends it early (the caller folds on one at a time).
HBW_FN double tie_double_folds(double v, double lo, double hi, double bottom, int& guard) {
  const double lo2 = 2.0 * lo, hi2 = 2.0 * hi, top = 2.0 * bottom;
  double x0 = v, xa = v, x1 = v;
  for (int n = 0; n < 4; ++n) {  // two settling folds, then the measured pair
    if (guard >= kGuard) return v;
    v = (v < lo ? lo2 : hi2) - v;
    ++guard;
    if (!(fabs(v) >= bottom && fabs(v) < top)) return v;
    if (n == 1) xa = v;
    if (n == 2) x1 = v;
  }
  (void)x0;
  int e;
  frexp(bottom, &e);
  const int eb = e - 1;
  const double scale = ldexp(1.0, 52 - eb);  // 1/g
  const double Ka = fabs(xa) * scale, K1 = fabs(x1) * scale, K2 = fabs(v) * scale;  // exact integers
  const double c1 = K1 - Ka, D = Ka - K2;
  if (!(D > 0.0) || !(K2 + (c1 > 0.0 ? c1 : 0.0) <= 0x1p53 - 2.0)) return v;
  const double n1 = K2 - 0x1p52 - 1.0, n2 = K2 + c1 - 0x1p52 - 1.0;
  if (!(n1 >= D) || !(n2 >= 0.0)) return v;
  double m = floor_div(n1, D);
  const double m2 = floor_div(n2, D) + 1.0;
  if (m2 < m) m = m2;
  const double cap = (double)((kGuard - guard) / 2);
  if (m > cap) m = cap;
  if (!(m >= 1.0)) return v;
  guard += 2 * (int)m;
  return copysign((K2 - m * D) * ldexp(1.0, eb - 52), v);
}

// v after the walls of one coordinate (flags: 1 reflecting, 2 periodic).
// Each pass: one fast-forward through the current binade, then single folds
// (a binade crossing, a rounding-tie binade, the last approach); the fold
// count and stopping rule are those of the plain loop.
HBW_FN double apply_wall(double v, double lo, double hi, double fl, double fh) {
  int guard = 0;
  if (fl == 1 && fh == 1) {
    const double lim2 = 2.0 * (fabs(lo) > fabs(hi) ? fabs(lo) : fabs(hi));
    const double lo2 = 2.0 * lo, hi2 = 2.0 * hi;  // exact
    // conditions combined with bitwise & / | (not && / ||): on a GPU lane each
    // short-circuit became its own exec-mask branch, ≈ 500 shader cycles per
    // trip of the fold loop below against ≈ 80 with one exit per trip
    // (scripts/wall_probe.py); the values and the fold count are the same
    while ((guard < kGuard) & ((v < lo) | (v > hi))) {
      int m, mode;
      double bottom;
      v = ff_double_folds(v, lo, hi, kGuard - guard, m, mode, bottom);
      guard += 2 * m;
      if (mode == kFfTie) {  // then fold on until the next binade
        v = tie_double_folds(v, lo, hi, bottom, guard);
        mode = kFfBinade;
      }
      // single folds (the plain loop's own steps): at least 4, then while
      // |v| > stop and fewer than smax.  After a fast-forward (v at the bottom
      // of its binade) or at a binade top, up to 16 take v below the next
      // binade edge by the fold reach 2 max(|lo|, |hi|), so the next pass can
      // fast-forward at once; a binade that cannot be fast-forwarded is folded
      // through (see ff_double_folds)
      const double edge = (mode == kFfDone ? bottom : 2.0 * bottom);
      const double stop = mode == kFfNear ? -1.0
                          : mode == kFfBinade ? bottom * (1.0 - 0x1p-53)  // |v| >= bottom
                                              : edge - lim2 - edge * 0x1p-48;
      const int smax = mode >= kFfBinade ? kGuard : 16;
      // the plain loop's folds, two per trip (predicated 4-fold groups for the
      // short runs measured 0.8 us per iteration slower): the second is taken under the
      // same test, so the sequence and the count are unchanged, and a GPU
      // lane pays one exec-mask branch per two dependent folds
      int s = 0;
      bool go = (guard < kGuard) & ((v < lo) | (v > hi)) & ((s < 4) | ((s < smax) & (fabs(v) > stop)));
      while (go) {
        const double v1 = (v < lo ? lo2 : hi2) - v;
        const bool two = (guard + 1 < kGuard) & ((v1 < lo) | (v1 > hi)) &
                         ((s + 1 < 4) | ((s + 1 < smax) & (fabs(v1) > stop)));
        v = two ? (v1 < lo ? lo2 : hi2) - v1 : v1;
        s += two ? 2 : 1;
        guard += two ? 2 : 1;
        go = two & (guard < kGuard) & ((v < lo) | (v > hi)) & ((s < 4) | ((s < smax) & (fabs(v) > stop)));
      }
    }
  } else {
    for (; guard < kGuard; ++guard) {
      const bool below = (fl == 1) & (v < lo);
      const bool above = (fh == 1) & (v > hi);
      if (!(below | above)) break;
      v = (v < lo) ? 2.0 * lo - v : 2.0 * hi - v;
    }
  }
  for (int g = 0; (fl == 2) & (v < lo) & (g < kGuard); ++g) v = hi + (v - lo);
  for (int g = 0; (fh == 2) & (v > hi) & (g < kGuard); ++g) v = lo + (v - hi);
  return v;
}

// the plain loop (reference order), for tests
HBW_FN double apply_wall_plain(double v, double lo, double hi, double fl, double fh) {
  for (int guard = 0; guard < kGuard; ++guard) {
    const bool below = (fl == 1) && (v < lo);
    const bool above = (fh == 1) && (v > hi);
    if (!(below || above)) break;
    v = (v < lo) ? 2.0 * lo - v : 2.0 * hi - v;
  }
  for (int g = 0; (fl == 2) && (v < lo) && g < kGuard; ++g) v = hi + (v - lo);
  for (int g = 0; (fh == 2) && (v > hi) && g < kGuard; ++g) v = lo + (v - hi);
  return v;
}

}  // namespace hbwall
