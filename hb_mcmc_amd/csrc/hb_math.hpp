// hb_math.hpp -- fp64 building blocks for the per-cadence hot loop on gfx950.
//
// The Kepler solve (likelihood3.c:152-166) evaluates sin/cos six times per
// cadence on an angle bounded by |E| < 2*pi + 1.  ocml's general sincos
// carries a Payne-Hanek branch and a 3-word reduction; here:
//   * reduction by x - n*pi/2 with a 2-word pi/2 and FMA (the first FMA is
//     exact for |n| < 2^20, so the reduced argument is correct to ~1 ulp);
//   * the fdlibm __kernel_sin/__kernel_cos minimax polynomials on
//     [-pi/4, pi/4] (< 1 ulp);
//   * quadrant selection with selects, no branches.
// Arguments outside |x| < 2^19 (never reached by the solver) or non-finite
// fall back to ocml's sincos.
//
// Division: v_rcp_f64 seed + two Newton steps + one residual correction
// (~1 ulp, no scaling fix-ups) for denominators known to be normal and
// O(1) -- Kepler's 1 - e cos E, the orbit's 1 - e cos E, 2*pi.
#pragma once
#include <hip/hip_runtime.h>

namespace hbdev {

// Wave votes on a lane predicate without materialising it as an int: HIP's
// __any/__all/__ballot take an int, so a compare result held as a lane mask
// is turned into 0/1 (v_cndmask) and back (v_cmp) -- two VALU instructions
// per vote.  The ballot builtin on a bool is a scalar AND with exec.
__device__ __forceinline__ unsigned long long wave_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0ull; }
__device__ __forceinline__ bool wave_all(bool p) {
  return __builtin_amdgcn_ballot_w64(p) == __builtin_amdgcn_ballot_w64(true);
}

// v_rcp_f64 is good to ~2^-24 (2.5e8 ulp, scripts/probes/rcp_probe.hip on
// the MI355X); one Newton step gives <= 11 ulp, two give the correctly
// rounded reciprocal on every probed input.
__device__ __forceinline__ double fast_rcp(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double r = fma(-d, y, 1.0);
  y = fma(r, y, y);
  r = fma(-d, y, 1.0);
  y = fma(r, y, y);
  return y;
}

// n / d for normal, moderate d (|d| in [2^-900, 2^900]).  Seed + ONE Newton
// step + the residual correction: the correction squares the quotient's
// error, and the probe found the result correctly rounded (== n / d) for all
// 4.2M inputs with d in [0.005, 2] -- the Kepler/orbit denominators.
__device__ __forceinline__ double fast_div(double n, double d) {
  double y = __builtin_amdgcn_rcp(d);
  y = fma(fma(-d, y, 1.0), y, y);
  const double q = n * y;
  return fma(fma(-d, q, n), y, q);
}

// sqrt(x) for x >= 0 in the normal range or 0: the v_rsq_f64 seed, one
// Goldschmidt step and the final residual correction (the sequence behind the
// library sqrt, without its denormal scaling and class fix-ups), within an
// ulp.  For square roots whose input is exact and whose output only needs a
// few ulp (the overlap area's sqrt(r^2 - h^2), asin's half-angle, the
// projected separation).
__device__ __forceinline__ double sqrt_fast(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y, h = 0.5 * y;
  const double r = fma(-s, h, 0.5);
  s = fma(s, r, s);
  h = fma(h, r, h);
  const double d = fma(-s, s, x);
  s = fma(d, h, s);
  return x == 0.0 ? 0.0 : s;  // rsq(0) = inf
}

// fdlibm kernels, |r| <= pi/4
__device__ __forceinline__ double ksin(double x, double z) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double r = fma(z, fma(z, fma(z, fma(z, S6, S5), S4), S3), S2);
  const double v = z * x;
  return fma(v, fma(z, r, S1), x);
}

__device__ __forceinline__ double kcos(double z) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double r = z * fma(z, fma(z, fma(z, fma(z, fma(z, C6, C5), C4), C3), C2), C1);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + z * r);
}

struct SinCos {
  double s, c;
};

// rare path (|x| >= 2^19 or non-finite): ocml, kept out of line so the
// hot loop's code stays small
__device__ __noinline__ SinCos sincos_ocml(double x) {
  SinCos r;
  sincos(x, &r.s, &r.c);
  return r;
}

// Branch-free fast path: valid for |x| < 2^19 (the caller checks the range
// once per wave and reruns out-of-range lanes through ocml).
__device__ __forceinline__ void sincos_fast(double x, double* s, double* c) {
  const double kInvPio2 = 6.36619772367581382433e-01;
  const double kPio2Hi = 1.57079632679489655800e+00;
  const double kPio2Lo = 6.12323399573676603587e-17;
  const double n = rint(x * kInvPio2);
  double r = fma(-n, kPio2Hi, x);
  r = fma(-n, kPio2Lo, r);
  const double z = r * r;
  const double sr = ksin(r, z);
  const double cr = kcos(z);
  const int q = (int)n;
  const bool swap = q & 1;
  double ss = swap ? cr : sr;
  double cc = swap ? sr : cr;
  if (q & 2) ss = -ss;
  if ((q + 1) & 2) cc = -cc;
  *s = ss;
  *c = cc;
}

__device__ __forceinline__ bool sincos_fast_ok(double x) { return fabs(x) < 524288.0; }

// (s, c) = (sin, cos)(E) -> (sin, cos)(E - d) for |d| <= 0.03 (Taylor to
// d^7 / d^8: truncation < 1e-19), by rotation: ~14 fp64 ops instead of a
// reduction + two kernels + quadrant select.
constexpr double kRotMax = 0.03;
__device__ __forceinline__ void rotate_back(double d, double& s, double& c) {
  const double z = d * d;
  const double sd = fma(d * z, fma(z, fma(z, -1.0 / 5040.0, 1.0 / 120.0), -1.0 / 6.0), d);
  const double cd = fma(z, fma(z, fma(z, fma(z, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5), 1.0);
  const double s2 = fma(s, cd, -c * sd);  // sin(E - d) = s cos d - c sin d
  const double c2 = fma(c, cd, s * sd);   // cos(E - d) = c cos d + s sin d
  s = s2;
  c = c2;
}

__device__ __forceinline__ void sincos_small(double x, double* s, double* c) {
  const double kInvPio2 = 6.36619772367581382433e-01;
  const double kPio2Hi = 1.57079632679489655800e+00;   // double(pi/2)
  const double kPio2Lo = 6.12323399573676603587e-17;   // pi/2 - kPio2Hi
  if (!(fabs(x) < 524288.0)) {  // 2^19; also NaN/inf
    const SinCos r = sincos_ocml(x);
    *s = r.s;
    *c = r.c;
    return;
  }
  const double n = rint(x * kInvPio2);
  double r = fma(-n, kPio2Hi, x);  // exact
  r = fma(-n, kPio2Lo, r);
  const double z = r * r;
  const double sr = ksin(r, z);
  const double cr = kcos(z);
  const int q = (int)n;
  const bool swap = q & 1;
  double ss = swap ? cr : sr;
  double cc = swap ? sr : cr;
  if (q & 2) ss = -ss;
  if ((q + 1) & 2) cc = -cc;
  *s = ss;
  *c = cc;
}

}  // namespace hbdev
