// hb_device.hpp -- device-side heartbeat-binary model for gfx950 (CDNA4).
//
// The reference evaluates, per walker and per cadence, ~120 libm calls
// (likelihood3.c:125-185 traj, :224-389 beaming/ellipsoidal/reflection/
// eclipse).  Almost all of them depend only on the walker's 21 parameters, so
// this file splits the model in two:
//
//   hb_prepare_walker()  -- once per walker: every mass/period/radius power,
//                           stellar tables, flux normalisation, beaming
//                           coefficients, the Gaia-G chi^2 term and the Roche
//                           flag, folded into one WalkerConst record.
//   hb_cadence_flux()    -- once per (walker, cadence): Kepler solve (5 Newton
//                           steps, exactly like likelihood3.c:160), true
//                           anomaly by the cos/sin form (no tan/atan), the
//                           2x3 photometric terms as a polynomial in
//                           beta = (1+e cos nu)/(1-e^2) and in the angle
//                           multiples of u = omega0+nu, and the eclipse.
//
// Arithmetic is fp64 throughout.  Results agree with the reference to a few
// ulp per cadence; the parity tolerance (1e-10 relative on logL) is stated in
// tests/test_gpu_parity.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hb_math.hpp"

namespace hbdev {

// physical constants, likelihood3.h:4-10
constexpr double kPi = 3.14159265358979323846;
constexpr double kTwoPi = 2.0 * 3.14159265358979323846;  // == 2*PI as a double
constexpr double kG = 6.6743e-8;
constexpr double kC = 2.998e10;
constexpr double kMsun = 1.9885e33;
constexpr double kRsun = 6.955e10;
constexpr double kDay = 86400.0;
constexpr double kBig = 1.e15;
constexpr int kNpars = 21;

// Per-walker record.  44 doubles = 352 B; read by the cadence kernel with
// wave-uniform (scalar) loads.
struct alignas(16) WalkerConst {
  // orbit (traj, likelihood3.c:125-185)
  double T0c;      // T0 [s]
  double Pc;       // P [s]
  double e;
  double e085;     // 0.85*e (initial Kepler guess, :157)
  double sq1me2;   // sqrt(1-e^2)
  double inv1me2;  // 1/(1-e^2)
  double cw, sw;   // cos/sin omega0
  double ci, si;   // cos/sin inc
  double aR;       // semi-major axis (traj's a) in Rsun
  // light-curve polynomial coefficients (both stars, Norm-weighted)
  double kconst;   // Norm1 + Norm2 + constant ellipsoidal term
  double kb;       // x cos u               (beaming)
  double kr0, kr2, krs;          // x beta^2 (1, cos2u, sin u)   (reflection)
  double kam2, kc21;             // x beta^3 (1, cos2u)
  double ks1, ks3;               // x beta^4 (sin u, sin3u)
  double kam3, kc22, kc4;        // x beta^5 (1, cos2u, cos4u)
  // eclipse (eclipse_area, :353-389); radii in Rsun, ordered big/small
  double ecl1, ecl2;             // Norm_k / (pi R_k^2)
  double rbig, rsml;             // unswapped R1, R2 are kept below
  double dcrit;                  // sqrt(Rbig^2 - Rsml^2)
  double r1, r2;
  // normalisation and scalar chi^2 pieces
  double blend, tune;
  double chi2_extra;             // ((Gmag - G_obs)/sigma_G)^2 (USE_GMAG=1)
  double roche;                  // 1.0 if RocheOverflow(), else 0.0
  double mA, mB;                 // mean anomaly M = fma(t, DAY, mB) * mA (hot loop)
  double rsum;                   // Rbig + Rsml
  // shared-period phase table (hb_prep_kernel): when this walker's period is
  // the batch's table period (tab = 1), sin/cos of the mean anomaly come from
  // the per-cadence table (sin, cos)(t DAY 2pi/P) rotated by psi = T0 2pi/P,
  // and those of the Kepler start E0 = M +- 0.85 e by a rotation through del
  double cpsi, spsi;             // cos/sin psi
  double cdel, sdel;             // cos/sin del, del = 0.85 e
  double tab;                    // 1.0: use the table, 0.0: direct sincos
  // cos/sin u numerators: cos u (1 - e cos E) = cw (cos E - e) - swq sin E,
  // sin u (1 - e cos E) = sw (cos E - e) + cwq sin E
  double swq, cwq;               // sin/cos omega0 x sqrt(1 - e^2)
  double ci2;                    // cos^2 inc
  double aR2, rsum2;             // aR^2, rsum^2 (the eclipse test dd aR^2 < rsum^2)
  double pad0;
};
static_assert(sizeof(WalkerConst) == 48 * 8, "WalkerConst layout");

// sqrt(1 - e^2) of the record, NaN at |e| = 1 as well as above: there the
// reference divides by 1 - e^2 = 0 (beta = (1 + e cos nu) / (1 - e^2) = 0 / 0,
// likelihood3.c:266, 326; the beaming factor's / sqrt(1 - e^2), :230) and its
// template is NaN, while the kernels' identity beta = 1 / (1 - e cos E) stays
// finite.  (e = 1 is also Roche overflow, periastron a (1 - e) = 0.)
__device__ __forceinline__ double sqrt_1me2(double e) {
  const double d = 1.0 - e * e;
  return d == 0.0 ? __builtin_nan("") : sqrt(d);
}

// logL mode: a walker whose logL is decided without its light curve.
//  * Roche overflow: chi^2 is replaced by 1e15 whatever the template is
//    (likelihood3.c:866-869): logL = -5e14.
//  * |e| >= 1 (the sampler puts no upper wall on e, likelihood3.c:986-1121, so
//    hot rungs propose it): sqrt(1 - e^2) is NaN (sqrt_1me2, |e| = 1
//    included), and with it every cadence's flux (traj, likelihood3.c:147-182),
//    the median, chi^2 and the reference's logL -- a NaN (+qNaN, what the
//    reference build returns for every such walker checked); a NaN logL is only
//    ever rejected by the Hastings test.
// Returns false when the light curve is needed.

__device__ __forceinline__ bool logl_without_light_curve(const WalkerConst& w, double& ll) {
  if (w.roche != 0.0) {
    ll = -kBig / 2.0;
    return true;
  }
  if (!(w.sq1me2 == w.sq1me2)) {
    ll = __builtin_nan("");
    return true;
  }
  return false;
}

// ------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------
__device__ __forceinline__ double sq(double x) { return x * x; }

// exact fmod(x, 2*PI) (fmod's result is always representable; fma with the
// right integer quotient reproduces it exactly).  Falls back to the libm
// routine for |x/2pi| >= 2^50, which folded light curves never reach.
__device__ __forceinline__ double fmod_twopi(double x) {
  const double y = kTwoPi;
  double q = trunc(x * 0.15915494309189533577);  // 1/(2 pi); off-by-one fixed below
  if (!(fabs(q) < 1125899906842624.0)) return fmod(x, y);  // 2^50 (also NaN/inf)
  double r = fma(-q, y, x);
  if (x >= 0.0) {
    if (r < 0.0) { q -= 1.0; r = fma(-q, y, x); }
    else if (r >= y) { q += 1.0; r = fma(-q, y, x); }
  } else {
    if (r > 0.0) { q += 1.0; r = fma(-q, y, x); }
    else if (r <= -y) { q -= 1.0; r = fma(-q, y, x); }
  }
  if (r == 0.0) r = copysign(0.0, x);
  return r;
}

// Branch-free fmod(x, 2*PI), exact for |x| < 2^19 (the caller checks the
// range and reruns other lanes through fmod_twopi).
__device__ __forceinline__ double fmod_twopi_fast(double x) {
  const double y = kTwoPi;
  double q = trunc(x * 0.15915494309189533577);
  const double r0 = fma(-q, y, x);
  const bool pos = x >= 0.0;
  double adj = 0.0;
  adj = (pos & (r0 < 0.0)) ? -1.0 : adj;
  adj = (pos & (r0 >= y)) ? 1.0 : adj;
  adj = (!pos & (r0 > 0.0)) ? 1.0 : adj;
  adj = (!pos & (r0 <= -y)) ? -1.0 : adj;
  q += adj;
  double r = fma(-q, y, x);
  r = (r == 0.0) ? copysign(0.0, x) : r;
  return r;
}

// sign(sin(M)) for M = fmod(., 2*PI) in (-2PI_d, 2PI_d), without a sine.
// PI_d < pi < nextafter(PI_d), so sin(M) > 0 exactly on (0, PI_d] and on
// (-2PI_d, -PI_d) (likelihood3.c:155-157 only uses the sign).
__device__ __forceinline__ double sign_sin_reduced(double m) {
  const double pos = (m <= kPi) ? 1.0 : -1.0;
  const double neg = (m < -kPi) ? 1.0 : -1.0;
  const double sg = (m > 0.0) ? pos : neg;
  return (m == 0.0) ? 0.0 : sg;
}

// order-preserving uint64 key of a double (non-NaN)
__device__ __forceinline__ uint64_t dkey(double v) {
  uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double dval(uint64_t k) {
  uint64_t b = (k & 0x8000000000000000ull) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

// ------------------------------------------------------------------------
// stellar tables (likelihood3.c:396-507); m is the linear mass in Msun
// ------------------------------------------------------------------------
__device__ __forceinline__ double logteff_of_mass(double m) {
  const double mn[16] = {0.1, 0.26, 0.47, 0.59, 0.69, 0.87, 0.98, 1.085,
                         1.4, 1.65, 2.0,  2.5,  3.0,  4.4,  15., 40.};
  const double tn[16] = {3.491, 3.531, 3.547, 3.584, 3.644, 3.712, 3.745, 3.774,
                         3.823, 3.863, 3.913, 3.991, 4.057, 4.182, 4.477, 4.623};
  if (m <= mn[0]) return tn[0];
  if (m >= mn[15]) return tn[15];
  double out = 0.0;
#pragma unroll
  for (int k = 15; k >= 1; --k)  // first node with m < mn[k], scanning up
    if (m < mn[k]) out = tn[k - 1] + (m - mn[k - 1]) * (tn[k] - tn[k - 1]) / (mn[k] - mn[k - 1]);
  return out;
}

__device__ __forceinline__ double logradius_of_mass(double m) {
  const double mn[10] = {0.07, 0.2, 0.356, 0.655, 0.784, 0.787, 1.377, 4.4, 15., 40.};
  const double rn[10] = {-0.953, -0.627, -0.423, -0.154, -0.082, -0.087, 0.295, 0.477, 0.792, 1.041};
  if (m <= mn[0]) return rn[0];
  if (m >= mn[9]) return rn[9];
  double out = __builtin_nan("");
#pragma unroll
  for (int k = 9; k >= 1; --k)
    if (m < mn[k]) out = rn[k - 1] + (m - mn[k - 1]) * (rn[k] - rn[k - 1]) / (mn[k] - mn[k - 1]);
  return out;
}

__device__ __forceinline__ double teff_spread() { return 0.0224; }  // envelope_Temp

__device__ __forceinline__ double radius_spread_of_mass(double m) {  // envelope_Radius
  const double ex = 4.22, sl = 15.68, lo = 0.01, knee = 1.055, hi = 0.17;
  return 1.0 / (1.0 / hi + 1.0 / (sl * pow(pow(m, ex) + pow(knee, ex), 1.0 / ex) - (sl * knee - lo)));
}
// the same law from lm = log10 m: m^ex = 10^(ex lm) does not wait for m = 10^lm
// (a few ulp from pow(10^lm, ex); the prep kernel's latency-critical chain)
__device__ __forceinline__ double radius_spread_of_logmass(double lm) {
  const double ex = 4.22, sl = 15.68, lo = 0.01, knee = 1.055, hi = 0.17;
  return 1.0 / (1.0 / hi + 1.0 / (sl * pow(exp10(ex * lm) + pow(knee, ex), 1.0 / ex) - (sl * knee - lo)));
}

// get_alpha_beam (likelihood3.c:194-209)
__device__ __forceinline__ double beam_coeff(double lt) {
  if (lt >= 4.5) return 1.2 / 4;
  if (lt < 3.5) return 6.5 / 4;
  double a0, a1, l0, l1;
  if (lt >= 3.9) { a0 = 2.5; a1 = 1.2; l0 = 3.9; l1 = 4.5; }
  else if (lt >= 3.7) { a0 = 4.0; a1 = 2.5; l0 = 3.7; l1 = 3.9; }
  else { a0 = 6.5; a1 = 4.0; l0 = 3.5; l1 = 3.7; }
  return (a1 + (a1 - a0) / (l1 - l0) * (lt - l1)) / 4;
}

// Stellar parameters from the 21-slot vector (calc_radii_and_Teffs).
struct Stellar {
  double m1, m2;          // Msun
  double r1, r2;          // Rsun
  double lt1, lt2;        // log10 Teff
  double t1, t2;          // K
};
__device__ __forceinline__ Stellar stellar_of(const double* p) {
  Stellar s;
  s.m1 = exp10(p[0]);
  s.m2 = exp10(p[1]);
  s.r1 = exp10(logradius_of_mass(s.m1) + p[7] * radius_spread_of_mass(s.m1));
  s.r2 = exp10(logradius_of_mass(s.m2) + p[8] * radius_spread_of_mass(s.m2));
  s.lt1 = logteff_of_mass(s.m1) + p[17] * teff_spread();
  s.lt2 = logteff_of_mass(s.m2) + p[18] * teff_spread();
  s.t1 = exp10(s.lt1);
  s.t2 = exp10(s.lt2);
  return s;
}

// Gaia-band (673 nm) magnitude of both stars (calc_mags, :725-795) and the
// full 4-band version for the C-ABI.  R in Rsun, T in K, dist in pc.
// one star's Planck factor of band_flux: pre / (exp(h nu / (k T)) - 1)
__device__ __forceinline__ double band_term(double lam_nm, double t) {
  const double hp = 6.626e-27, kb = 1.38e-16;
  double fr = kC / (lam_nm * 1e-7);
  double pre = 2.0 * hp * (fr * fr * fr) / (kC * kC);
  return pre / (exp(hp * fr / (kb * t)) - 1.0);
}
// band_flux from both stars' Planck factors (the prep computes each in the
// wave that has its star's temperature)
__device__ __forceinline__ double band_flux_terms(double r1cm, double r2cm, double bt1, double bt2, double dist,
                                                  double blend) {
  const double pc = 3.086e18;
  double f = kPi * (r1cm * r1cm * bt1 + r2cm * r2cm * bt2) / ((dist * dist) * (pc * pc));
  return f / (1.0 - blend);
}
__device__ __forceinline__ double band_flux(double lam_nm, double r1cm, double r2cm, double t1,
                                            double t2, double dist, double blend) {
  return band_flux_terms(r1cm, r2cm, band_term(lam_nm, t1), band_term(lam_nm, t2), dist, blend);
}
__device__ __forceinline__ double ab_mag(double f) { return -2.5 * log10(f) - 48.6; }

// Eggleton 1983 Roche-lobe radius over separation (likelihood3.c:945-948)
__device__ __forceinline__ double lobe_fraction(double q) {
  double c = cbrt(q);
  double c2 = c * c;
  return 0.49 * c2 / (0.6 * c2 + log(1.0 + c));
}

// ------------------------------------------------------------------------
// per-star photometric coefficients (beaming :224-236, ellipsoidal :255-307,
// reflection :322-337) with every cadence-independent factor hoisted:
//   beaming     = kb * cos u
//   ellipsoidal = am1 + b^3 (am2 + c21 cos2u) + b^4 (s1 sin u + s3 sin3u)
//                     + b^5 (am3 + c22 cos2u + c4 cos4u)
//   reflection  = kref * b^2 * (0.64 - sin i sin u + 0.18 sin^2 i (1 - cos2u))
// with b = (1 + e cos nu)/(1 - e^2) and u = omega + nu.
// ------------------------------------------------------------------------
struct StarCoef {
  double kb, am1, am2, c21, am3, c22, c4, s1, s3, kref;
};

// star_coef in three steps, for the prep's lane layout: star_coef_x holds
// everything that needs neither radius (the factors in front of each
// coefficient's R^k), star_coef_r multiplies the star's own radius in, and
// star_coef_finish the companion's radius (reflection) and alpha_beam
// (beaming).  Each coefficient's operations and their order are those of the
// one-expression form (left to right: the R^k factor and ppm come last), except
// the beaming coefficient kb: alpha_beam comes from another prep wave, so it
// multiplies the product last instead of second (likelihood3.c:233 has
// -2830 * alpha_beam * ...): an ulp-level difference, well inside the template
// tolerance (the reference's per-cadence product, fac4 included, is hoisted
// here anyway).
struct StarCoefX {
  double kb, am1, am2, c21, a3, a22, a4, x5, b1, b3, x4, kref;
};
__device__ __forceinline__ StarCoefX star_coef_x(double pd, double ma, double mb, double e, double si, double mu,
                                                 double tau, double aref) {
  const double ppm = 1.e-6;
  const double s2 = si * si, s3 = s2 * si, s4 = s3 * si;
  const double cP = cbrt(pd);
  const double inv_pd = 1.0 / pd;
  const double omE = 1.0 - e;
  const double prot = pd * (omE * sqrt(omE));  // P (1-e)^{3/2}
  const double q = mb / ma;
  const double opq = 1.0 + q;
  const double cM = cbrt(ma);
  const double cq = cbrt(opq);
  const double inv_ma = 1.0 / ma;
  StarCoefX x;
  // beaming: pow(1+q, 2/3) is integer 2/3 == 0 in the reference -> factor 1
  x.kb = -2830. * q * cM / cP * si / sqrt(1.0 - e * e) * ppm;
  const double a11 = 15 * mu * (2 + tau) / (32 * (3 - mu));
  const double a21 = 3 * (15 + mu) * (1 + tau) / (20 * (3 - mu));
  const double a2b = 15 * (1 - mu) * (3 + tau) / (64 * (3 - mu));
  const double a01 = a21 / 9, a0b = 3 * a2b / 20, a31 = 5 * a11 / 3, a41 = 7 * a2b / 4;
  const double qq = q / opq;
  x.am1 = 26870 * a01 * (2 - 3 * s2) * inv_ma / (prot * prot);
  x.am2 = 40305 * a01 * (2 - 3 * s2) * inv_ma * qq * (inv_pd * inv_pd);
  x.c21 = 13435 * a21 * s2 * inv_ma * qq * (inv_pd * inv_pd);
  // M^-5/3 q/(1+q)^5/3 P^-10/3 (x R^5 ppm)
  x.x5 = qq / (cq * cq) * inv_ma / (cM * cM) * (inv_pd * inv_pd * inv_pd) / cP;
  x.a3 = 759 * a0b * (8 - 40 * s2 + 35 * s4);
  x.a22 = 759 * a2b * (6 * s2 - 7 * s4);
  x.a4 = 759 * a41 * s4;
  // M^-4/3 q/(1+q)^4/3 P^-8/3 (x R^4 ppm)
  x.x4 = qq / cq * inv_ma / cM * (inv_pd * inv_pd) / (cP * cP);
  x.b1 = 3194 * a11 * (4 * si - 5 * s3);
  x.b3 = 3194 * a31 * s3;
  // reflection: (1+q)^-2/3 M^-2/3 P^-4/3 (Rc^2 ppm: star_coef_finish)
  x.kref = 56514 * aref / (cq * cq) / (cM * cM) * inv_pd / cP;
  return x;
}
__device__ __forceinline__ StarCoef star_coef_r(const StarCoefX& x, double rk) {
  const double ppm = 1.e-6;
  const double rk3 = rk * rk * rk;
  StarCoef c;
  c.kb = x.kb;
  c.am1 = x.am1 * rk3 * ppm;
  c.am2 = x.am2 * rk3 * ppm;
  c.c21 = x.c21 * rk3 * ppm;
  const double c5 = x.x5 * (rk3 * rk * rk) * ppm;
  c.am3 = x.a3 * c5;
  c.c22 = x.a22 * c5;
  c.c4 = x.a4 * c5;
  const double c4c = x.x4 * (rk3 * rk) * ppm;
  c.s1 = x.b1 * c4c;
  c.s3 = x.b3 * c4c;
  c.kref = x.kref;
  return c;
}
__device__ __forceinline__ StarCoef star_coef_pre(double pd, double ma, double mb, double e, double si,
                                                  double rk, double mu, double tau, double aref) {
  return star_coef_r(star_coef_x(pd, ma, mb, e, si, mu, tau, aref), rk);
}
__device__ __forceinline__ void star_coef_finish(StarCoef& c, double rc, double ab) {
  const double ppm = 1.e-6;
  c.kb = ab * c.kb;
  c.kref = c.kref * (rc * rc) * ppm;
}
__device__ __forceinline__ StarCoef star_coef(double pd, double ma, double mb, double e, double si,
                                              double rk, double rc, double mu, double tau,
                                              double aref, double ab) {
  StarCoef c = star_coef_pre(pd, ma, mb, e, si, rk, mu, tau, aref);
  star_coef_finish(c, rc, ab);
  return c;
}

// ------------------------------------------------------------------------
// per-walker preparation
// ------------------------------------------------------------------------
// The polynomial's harmonics in x = sin^2 u: cos 2u = 1 - 2x,
// cos 4u = 1 - 8x + 8x^2, sin 3u = sin u (3 - 4x), so each beta-power's
// coefficient is a polynomial in x (sin u) with the harmonic weights folded
// into the record once per walker: 8 fp64 instructions per cadence instead of
// 13.  The record's k* fields hold the x-form (su2_form).
//
// the cos-harmonic coefficients (kr0, kr2 | kam2, kc21 | ks1, ks3 | kam3,
// kc22, kc4 of 1, cos 2u, sin u, sin 3u, cos 4u) rewritten as polynomials in
// x = sin^2 u
__host__ __device__ inline void su2_form(double& kr0, double& kr2, double& kam2, double& kc21, double& ks1, double& ks3,
                                         double& kam3, double& kc22, double& kc4) {
  kr0 = kr0 + kr2;  // kr0 + kr2 (1 - 2x)
  kr2 = -2.0 * kr2;
  kam2 = kam2 + kc21;  // kam2 + kc21 (1 - 2x)
  kc21 = -2.0 * kc21;
  ks1 = fma(3.0, ks3, ks1);  // sin u (ks1 + ks3 (3 - 4x))
  ks3 = -4.0 * ks3;
  kam3 = (kam3 + kc22) + kc4;  // kam3 + kc22 (1 - 2x) + kc4 (1 - 8x + 8x^2)
  kc22 = fma(-8.0, kc4, -2.0 * kc22);
  kc4 = 8.0 * kc4;
}

__device__ inline void hb_prepare_walker(const double* __restrict__ p, const double* __restrict__ mag,
                                         const double* __restrict__ magerr, WalkerConst& w) {
  const double pd = exp10(p[2]);          // period [d]
  const double e = p[3], inc = p[4], om = p[5];
  const Stellar st = stellar_of(p);
  const double m1 = st.m1, m2 = st.m2;

  // orbit
  w.Pc = pd * kDay;
  w.T0c = p[6] * kDay;
  w.e = e;
  w.e085 = 0.85 * e;
  w.sq1me2 = sqrt_1me2(e);
  w.inv1me2 = 1.0 / (1.0 - e * e);
  sincos(om, &w.sw, &w.cw);
  double si, ci;
  sincos(inc, &si, &ci);
  w.si = si;
  w.ci = ci;
  const double mtot_cgs = m1 * kMsun + m2 * kMsun;
  const double a_cgs = cbrt(kG * mtot_cgs * (w.Pc * w.Pc) / (kTwoPi * kTwoPi));
  w.aR = a_cgs / kRsun;

  // flux normalisation (calc_light_curve :613-614)
  const double l1 = sq(st.r1) * sq(sq(st.t1));
  const double l2 = sq(st.r2) * sq(sq(st.t2));
  const double n1 = l1 / (l1 + l2);
  const double n2 = l2 / (l1 + l2);

  // beaming coefficients (:619-624); log10(Teff) is the table value itself
  const double ab1 = beam_coeff(st.lt1) * exp(p[15]);
  const double ab2 = beam_coeff(st.lt2) * exp(p[16]);

  const StarCoef c1 = star_coef(pd, m1, m2, e, si, st.r1, st.r2, p[9], p[10], p[13], ab1);
  const StarCoef c2 = star_coef(pd, m2, m1, e, si, st.r2, st.r1, p[11], p[12], p[14], ab2);

  // star 2 sees u+pi: odd harmonics of u flip sign
  const double s2 = si * si;
  w.kconst = n1 + n2 + (n1 * c1.am1 + n2 * c2.am1);
  w.kb = n1 * c1.kb - n2 * c2.kb;
  const double rp = n1 * c1.kref + n2 * c2.kref;
  const double rm = n1 * c1.kref - n2 * c2.kref;
  w.kr0 = rp * (0.64 + 0.18 * s2);
  w.kr2 = -rp * (0.18 * s2);
  w.krs = -rm * si;
  w.kam2 = n1 * c1.am2 + n2 * c2.am2;
  w.kc21 = n1 * c1.c21 + n2 * c2.c21;
  w.ks1 = n1 * c1.s1 - n2 * c2.s1;
  w.ks3 = n1 * c1.s3 - n2 * c2.s3;
  w.kam3 = n1 * c1.am3 + n2 * c2.am3;
  w.kc22 = n1 * c1.c22 + n2 * c2.c22;
  w.kc4 = n1 * c1.c4 + n2 * c2.c4;
  su2_form(w.kr0, w.kr2, w.kam2, w.kc21, w.ks1, w.ks3, w.kam3, w.kc22, w.kc4);

  // eclipse
  w.r1 = st.r1;
  w.r2 = st.r2;
  w.ecl1 = n1 / (kPi * (st.r1 * st.r1));
  w.ecl2 = n2 / (kPi * (st.r2 * st.r2));
  w.rbig = st.r2 > st.r1 ? st.r2 : st.r1;
  w.rsml = st.r2 > st.r1 ? st.r1 : st.r2;
  w.dcrit = sqrt(w.rbig * w.rbig - w.rsml * w.rsml);

  w.blend = p[19];
  w.tune = p[20];

  // Gaia G term (loglikelihood :834-848), only the 673 nm band is used
  const double g = ab_mag(band_flux(673.0, st.r1 * kRsun, st.r2 * kRsun, st.t1, st.t2, mag[0], p[19]));
  const double gr = (g - mag[1]) / magerr[0];
  w.chi2_extra = gr * gr;

  // Roche overflow (:953-974), separation from the same Kepler a
  const double q12 = m1 / m2;
  const double peri = a_cgs * (1.0 - e);
  const double f1 = (st.r1 * kRsun) / peri;
  const double f2 = (st.r2 * kRsun) / peri;
  w.roche = ((lobe_fraction(q12) < f1) || (lobe_fraction(1.0 / q12) < f2)) ? 1.0 : 0.0;
  // hot-loop mean anomaly: (t DAY - T0 DAY) * (2 pi / P), two roundings
  // like the reference's three (likelihood3.c:149-152)
  w.mA = kTwoPi / w.Pc;
  w.mB = -w.T0c;
  w.rsum = w.rbig + w.rsml;
  w.cpsi = 1.0;
  w.spsi = 0.0;
  w.cdel = 1.0;
  w.sdel = 0.0;
  w.tab = 0.0;  // the scalar drop-in paths evaluate sin/cos directly
  w.swq = w.sw * w.sq1me2;
  w.cwq = w.cw * w.sq1me2;
  w.ci2 = w.ci * w.ci;
  w.aR2 = w.aR * w.aR;
  w.rsum2 = w.rsum * w.rsum;
  w.pad0 = 0.0;
}

// ------------------------------------------------------------------------
// eclipse_area (likelihood3.c:353-389) with pre-ordered radii (Rsun), d>=0
// ------------------------------------------------------------------------
// asin on [0, 1] (the chord angles hh / r of the overlap area): asin(s) =
// s + s t P(t), t = s^2, for s < 0.5, and asin(x) = pi/2 - 2 asin(sqrt((1 - x) / 2))
// above (the halving is exact there).  P is a degree-12 Chebyshev fit on
// [0, 1/4] (scripts/fit_asin.py: fit error 1.5e-17; the float64 evaluation is
// within 2 ulp of asin over [0, 1]).  Branch-free, because one eclipse flush
// mixes lanes of both ranges; ~35 instructions against ~95 for ocml's asin,
// whose two calls were a third of the eclipse flush.  x > 1 (hh rounded past
// r) and NaN give NaN, like libm.
__device__ __forceinline__ double asin01(double x) {
  const bool big = x >= 0.5;
  const double t = big ? (1.0 - x) * 0.5 : x * x;
  const double s = big ? sqrt_fast(t) : x;  // t exact (Sterbenz); a few ulp of s are within asin01's 2 ulp
  double p = 0.028757851367421566;
  p = __builtin_fma(p, t, -0.014851887071247204);
  p = __builtin_fma(p, t, 0.01740087944269402);
  p = __builtin_fma(p, t, 0.005457506718640358);
  p = __builtin_fma(p, t, 0.01032281435018578);
  p = __builtin_fma(p, t, 0.011479177415184906);
  p = __builtin_fma(p, t, 0.013971212973552933);
  p = __builtin_fma(p, t, 0.017352392720869973);
  p = __builtin_fma(p, t, 0.02237217294214989);
  p = __builtin_fma(p, t, 0.030381944138531247);
  p = __builtin_fma(p, t, 0.04464285714635543);
  p = __builtin_fma(p, t, 0.07499999999998433);
  p = __builtin_fma(p, t, 0.16666666666666669);
  const double r = __builtin_fma(s * t, p, s);
  return big ? (1.5707963267948966 - 2.0 * r) + 6.123233995736766e-17 : r;
}

__device__ __forceinline__ double overlap_partial(double ra, double rb, double d, bool inner) {
  const double cq = d * d - rb * rb + ra * ra;
  const double hh = sqrt((4. * d * d * ra * ra - cq * cq) / (4. * d * d));
  // hh and the chord ratios keep the reference's IEEE operations (asin's slope
  // is unbounded at hh = rb); sqrt(r^2 - hh^2) only needs its output to an ulp
  const double la = ra * ra * asin01(hh / ra) - hh * sqrt_fast(ra * ra - hh * hh);
  const double lb = rb * rb * asin01(hh / rb) - hh * sqrt_fast(rb * rb - hh * hh);
  return inner ? (kPi * rb * rb - (-la + lb)) : (la + lb);
}

__device__ __forceinline__ double overlap_area(double ra, double rb, double dc, double d) {
  double area = 0.0;
  if (d < ra - rb) area = kPi * rb * rb;
  const bool outer = (d > dc) & (d < ra + rb);
  const bool inner = (d <= dc) & (d >= ra - rb);
  if (outer | inner) area = overlap_partial(ra, rb, d, inner);
  return area;
}

// area * Norm_k / (pi R_k^2) for the star in front; out of line (rare)
__device__ __noinline__ double eclipse_term(const WalkerConst* w, double dR, double zz) {
  const double area = overlap_area(w->rbig, w->rsml, w->dcrit, dR);
  return area * (zz < 0.0 ? w->ecl2 : w->ecl1);
}
// the same, inlined (the deferred queue applies it after the model loop)
__device__ __forceinline__ double eclipse_term_inl(const WalkerConst* w, double dR, double zz) {
  const double area = overlap_area(w->rbig, w->rsml, w->dcrit, dR);
  return area * (zz < 0.0 ? w->ecl2 : w->ecl1);
}

// ------------------------------------------------------------------------
// one cadence: returns Amag1 + Amag2 before median removal
// ------------------------------------------------------------------------
struct Orbit {
  double cu, su;   // cos/sin(omega0 + nu)
  double beta;     // (1 + e cos nu)/(1 - e^2)
  double dR;       // projected separation [Rsun]
  double zz;       // sign carrier of Z1 - Z2 (>0: star 1 in front)
  double rR;       // radial separation [Rsun]
  double cnu, snu; // cos/sin nu
};

__device__ __forceinline__ Orbit hb_orbit(double t, const WalkerConst& w) {
  const double e = w.e;
  double m = kTwoPi * (t * kDay - w.T0c) / w.Pc;
  m = fmod_twopi(m);
  const double sg = sign_sin_reduced(m);
  double E = (sg == 0.0) ? m : m + w.e085 * sg;
  double s, c;
#pragma unroll
  for (int it = 0; it < 5; ++it) {
    sincos_small(E, &s, &c);
    E = E - ((E - e * s) - m) / (1.0 - e * c);
  }
  sincos_small(E, &s, &c);
  const double den = 1.0 - e * c;
  const double inv = 1.0 / den;
  Orbit o;
  o.cnu = (c - e) * inv;
  o.snu = w.sq1me2 * s * inv;
  o.cu = w.cw * o.cnu - w.sw * o.snu;
  o.su = w.sw * o.cnu + w.cw * o.snu;
  o.beta = (1.0 + e * o.cnu) * w.inv1me2;
  o.rR = w.aR * den;
  const double sci = o.su * w.ci;
  o.dR = o.rR * sqrt(o.cu * o.cu + sci * sci);
  o.zz = o.su * w.si;
  return o;
}

__device__ __noinline__ double hb_cadence_flux_slow(double t, const WalkerConst* w);

__device__ __forceinline__ double hb_cadence_flux(double t, const WalkerConst& w) {
  const Orbit o = hb_orbit(t, w);
  const double cu = o.cu, su = o.su;
  const double b = o.beta;
  const double b2 = b * b;
  const double b3 = b2 * b;
  double v = w.kconst + w.kb * cu;
  const double x = su * su;  // the record's harmonics in x = sin^2 u (su2_form)
  v += b2 * (w.kr0 + w.kr2 * x + w.krs * su);
  v += b3 * (w.kam2 + w.kc21 * x);
  v += (b2 * b2) * (su * (w.ks1 + w.ks3 * x));
  v += (b3 * b2) * (w.kam3 + x * (w.kc22 + w.kc4 * x));
  // eclipse: only lanes with overlap take the branch
  if (o.dR < w.rbig + w.rsml && o.zz != 0.0) {
    const double area = overlap_area(w.rbig, w.rsml, w.dcrit, o.dR);
    v -= area * (o.zz < 0.0 ? w.ecl2 : w.ecl1);
  }
  return v;
}

// reference-order path for lanes outside the fast sincos/fmod domain
__device__ __noinline__ double hb_cadence_flux_slow(double t, const WalkerConst* w) {
  return hb_cadence_flux(t, *w);
}

// ------------------------------------------------------------------------
// K cadences at once, branch-free: the K Kepler chains interleave in one
// basic block (ILP for the fp64 dependency chains).  Lanes whose angles
// leave the fast sincos/fmod domain set `bad`; the caller reruns them
// through hb_cadence_flux (ocml path) under one wave-uniform branch.
//
// Mean anomaly: q = trunc(x / 2pi), r = x - q 2pi by one FMA.  When q is the
// true quotient r IS fmod(x, 2pi) (exact), and r lies strictly inside
// (0, 2pi) on x's side; an off-by-one q lands r on or outside that interval
// (FMA rounding is monotone), so those lanes -- and r == 0, where the sign of
// zero matters -- take fmod_twopi_fast under a wave-uniform branch.
//
// Newton on E - e sin E = M (likelihood3.c:160): the reference always takes
// 5 steps; here the wave leaves the loop once every lane's predicted next
// correction e d^2 / (2 (1 - e cos E)) is below a quarter ulp of E (2^-54
// |E|), i.e. the remaining steps would only move E by rounding noise (the parity budget is 1e-12 on the template).  e = 0.23 (the C2 workload)
// converges in 3 steps, e -> 0.99 keeps all 5.  The step uses the v_rcp_f64
// seed with one Newton refinement (relative error ~2^-48, which only scales
// the step and is absorbed by the next one); (sin, cos) follow E by rotation
// through the step (Taylor to d^11 / d^12, truncation < 3e-18 for |d| <= 0.25)
// (fewer terms when the wave's steps are below 2^-9 / 2^-22) when the whole
// wave's steps are small, else by direct evaluation.
// The light-curve polynomial is written with explicit FMAs (the build uses
// -ffp-contract=off so that the reference-order paths keep their rounding).
// ------------------------------------------------------------------------
constexpr double kRotMaxK = 0.25;
__device__ __forceinline__ void rotate_back_wide(double d, double z, double& s, double& c) {
  // sin d = d (1 + z S(z)), cos d = 1 + z C(z), z = d^2
  const double sp = z * fma(z, fma(z, fma(z, fma(z, -1.0 / 39916800.0, 1.0 / 362880.0), -1.0 / 5040.0),
                                 1.0 / 120.0), -1.0 / 6.0);
  const double sd = fma(d, sp, d);
  const double cd = fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, 1.0 / 479001600.0, -1.0 / 3628800.0),
                                                        1.0 / 40320.0), -1.0 / 720.0), 1.0 / 24.0), -0.5),
                        1.0);
  const double s2 = fma(s, cd, -c * sd);  // sin(E - d) = s cos d - c sin d
  const double c2 = fma(c, cd, s * sd);   // cos(E - d) = c cos d + s sin d
  s = s2;
  c = c2;
}
// |d| <= 2^-9: Taylor to d^5 / d^4 (truncation < 8e-20)
__device__ __forceinline__ void rotate_back_mid(double d, double z, double& s, double& c) {
  const double sd = fma(d, z * fma(z, 1.0 / 120.0, -1.0 / 6.0), d);
  const double cd = fma(z, fma(z, 1.0 / 24.0, -0.5), 1.0);
  const double s2 = fma(s, cd, -c * sd);
  const double c2 = fma(c, cd, s * sd);
  s = s2;
  c = c2;
}
// |d| <= 2^-22: sin d = d, cos d = 1 - d^2/2 (truncation < 3e-21)
__device__ __forceinline__ void rotate_back_tiny(double d, double z, double& s, double& c) {
  const double cd = fma(z, -0.5, 1.0);
  const double s2 = fma(s, cd, -c * d);
  const double c2 = fma(c, cd, s * d);
  s = s2;
  c = c2;
}

// Mean anomaly of K cadences: q = trunc(x / 2pi), r = x - q 2pi (exact when
// q is the true quotient, see above); `exact` flags lanes that need
// fmod_twopi_fast, `ok` lanes inside the fast sincos/fmod domain, plus[k] =
// sign(sin m) > 0 (sign_sin_reduced for m in (-2pi, 2pi) \ {0}).
template <int K>
__device__ __forceinline__ void mean_anomaly_k(const double (&t)[K], const WalkerConst& w, double (&m)[K],
                                               bool (&plus)[K], bool& ok, bool& exact) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double x = fma(t[k], kDay, w.mB) * w.mA;
    ok &= sincos_fast_ok(x);
    const double q = trunc(x * 0.15915494309189533577);
    const double r = fma(-q, kTwoPi, x);
    // r != 0, |r| < 2pi and sign(r) == sign(x), branch-free
    const bool same_sign = (__double_as_longlong(r) ^ __double_as_longlong(x)) >= 0;
    const bool inside = same_sign & (fabs(r) < kTwoPi) & (r != 0.0);
    exact |= !inside;
    m[k] = r;
    plus[k] = (fabs(r) <= kPi) != (r < 0.0);
  }
}

// The reference's Kepler start E0 = M + 0.85 e sign(sin M) (likelihood3.c:
// 155-157) and (sin, cos)(E0): rotations of the shared-period table entry
// (tab), else the branch-free sincos.  Lanes flagged `exact` recompute M by
// fmod_twopi_fast first (wave-uniform branch).
//
// Series start (tab and |e| <= kSeriesEmax): E0 = M + the fifth-order Lagrange
// series of Kepler's equation in e, written in s = sin M, c = cos M, x = s^2:
//   E - M = s [c ((e^2 + e^4) - 8/3 e^4 x)
//              + (e + e^3 + e^5) + x (-(3/2 e^3 + 17/3 e^5) + 125/24 e^5 x)] + O(e^6)
// (e sin M + e^2/2 sin 2M + e^3/8 (3 sin 3M - sin M) + e^4/6 (2 sin 4M - sin 2M)
// + e^5/384 (125 sin 5M - 81 sin 3M + 2 sin M)), and (sin, cos)(E0) by the
// Taylor rotation of the table entry through E0 - M (|E0 - M| <= e + O(e^6)
// <= kRotMaxK).  The start is within 8e-5 of the root at e = 0.226 (1.5e-4 at
// 0.25), so Newton converges in two steps where the reference's start takes
// three (scripts/kepler_series.py); for e <= 0.85 every start Newton
// converges from reaches the reference's root to rounding
// (scripts/kepler_warm.py), so only the path there changes.
#ifndef HB_SERIES_EMAX
#define HB_SERIES_EMAX 0.25  // A/B knob (0: the reference's start everywhere)
#endif
constexpr double kSeriesEmax = HB_SERIES_EMAX;
static_assert(kSeriesEmax <= kRotMaxK, "the series start's rotation needs |E0 - M| <= kRotMaxK");
template <int K>
__device__ __forceinline__ void cold_start_k(const double (&t)[K], const double2 (&ph)[K], bool tab, bool exact,
                                             const WalkerConst& w, double (&m)[K], const bool (&plus)[K],
                                             double (&E)[K], double (&s)[K], double (&c)[K], bool& ok) {
  const bool ser = tab && fabs(w.e) <= kSeriesEmax;  // walker-uniform
  if (ser) {
    const double e = w.e, e2 = e * e, e3 = e2 * e, e4 = e2 * e2, e5 = e4 * e;
    const double a0 = e2 + e4, a1 = (-8.0 / 3.0) * e4;
    const double b0 = (e + e3) + e5, b1 = -(1.5 * e3 + (17.0 / 3.0) * e5), b2 = (125.0 / 24.0) * e5;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double sx = fma(ph[k].x, w.cpsi, -(ph[k].y * w.spsi));  // sin M
      const double cx = fma(ph[k].y, w.cpsi, ph[k].x * w.spsi);     // cos M
      const double x = sx * sx;
      const double dl = sx * fma(cx, fma(x, a1, a0), fma(x, fma(x, b2, b1), b0));
      E[k] = m[k] + dl;
      s[k] = sx;
      c[k] = cx;
      rotate_back_wide(-dl, dl * dl, s[k], c[k]);  // (sin, cos)(M + dl)
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) E[k] = m[k] + (plus[k] ? w.e085 : -w.e085);
  }
  if (tab && !ser) {  // walker-uniform: E0 = M + sg del by rotations of the table entry
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double sx = fma(ph[k].x, w.cpsi, -(ph[k].y * w.spsi));  // sin(phi - psi)
      const double cx = fma(ph[k].y, w.cpsi, ph[k].x * w.spsi);     // cos(phi - psi)
      const double sd = plus[k] ? w.sdel : -w.sdel;
      s[k] = fma(sx, w.cdel, cx * sd);
      c[k] = fma(cx, w.cdel, -(sx * sd));
    }
  }
  if (wave_any(exact)) {  // rare: x near a multiple of 2pi, or r == 0
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double x = fma(t[k], kDay, w.mB) * w.mA;
      m[k] = fmod_twopi_fast(x);
      const double sg = sign_sin_reduced(m[k]);
      E[k] = (sg == 0.0) ? m[k] : m[k] + w.e085 * sg;
    }
    tab = false;  // recompute (s, c) directly below
  }
  if (!tab) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      ok &= sincos_fast_ok(E[k]);
      sincos_fast(E[k], &s[k], &c[k]);
    }
  }
}

// Newton on E - e sin E = M (likelihood3.c:152-160), at most 5 steps; the
// wave leaves once every lane's predicted next correction is <= 2^-54 |E| (a
// quarter ulp of E).
// yk: the last step's 1/(1 - e cos E).  Returns whether it converged.
template <int K>
__device__ __forceinline__ bool newton_k(double e, const double (&m)[K], double (&E)[K], double (&s)[K],
                                         double (&c)[K], double (&yk)[K], bool& ok) {
  const double ae53 = 0x1p53 * fabs(e);
#pragma unroll
  for (int it = 0; it < 5; ++it) {
    bool small = true, mid = true, tiny = true, conv = true;
    double d[K], z[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double den = fma(-e, c[k], 1.0);
      double y = __builtin_amdgcn_rcp(den);
      y = fma(fma(-den, y, 1.0), y, y);
      yk[k] = y;
      d[k] = ((E[k] - e * s[k]) - m[k]) * y;
      E[k] = E[k] - d[k];
      z[k] = d[k] * d[k];
      const double ad = fabs(d[k]);
      small &= ad <= kRotMaxK;
      mid &= ad <= 0x1p-9;
      tiny &= ad <= 0x1p-22;
      // |e|: e < 0 is Kepler's equation at M + pi.  The predicted next
      // correction e d^2 / (2 den) at most 2^-54 |E|, a quarter ulp of E (the
      // absolute 2^-52 of rounds 1-5 left up to 2.8 ulp of E at |E| < 1,
      // tests/test_gpu_parity.py::test_kepler_cold_start_against_reference_
      // root); as many multiplies as that rule (2^53 |e| hoisted)
      conv &= ae53 * z[k] <= den * fabs(E[k]);
    }
    // rotation degree by the wave's largest step (wave-uniform branches)
    if (wave_all(tiny)) {
#pragma unroll
      for (int k = 0; k < K; ++k) rotate_back_tiny(d[k], z[k], s[k], c[k]);
    } else if (wave_all(mid)) {
#pragma unroll
      for (int k = 0; k < K; ++k) rotate_back_mid(d[k], z[k], s[k], c[k]);
    } else if (wave_all(small)) {
#pragma unroll
      for (int k = 0; k < K; ++k) rotate_back_wide(d[k], z[k], s[k], c[k]);
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        ok &= sincos_fast_ok(E[k]);
        sincos_fast(E[k], &s[k], &c[k]);
      }
    }
    if (wave_all(conv)) return true;
  }
  return false;
}

// The photometric polynomial of K cadences from (sin, cos) of the solved
// eccentric anomaly and inv[k] = 1 / (1 - e cos E), without the eclipse;
// dd = (projected separation / a)^2 and zz (sign carrier of Z1 - Z2) for the
// eclipse test.  u = omega0 + nu from the numerators of cos/sin nu (den > 0):
// cos u (1 - e cos E) = cw (cos E - e) - sw sqrt(1-e^2) sin E, likewise sin u;
// beta = (1 + e cos nu) / (1 - e^2) = 1 / (1 - e cos E) identically, and the
// squared projected separation / a^2 is CU^2 + cos^2 i SU^2 (no atan/tan).
template <int K>
__device__ __forceinline__ void flux_poly_inv_k(const double (&s)[K], const double (&c)[K], const double (&invk)[K],
                                                const WalkerConst& w, double (&v)[K], double (&dd)[K],
                                                double (&zz)[K]) {
  const double e = w.e;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double inv = invk[k];
    const double P = c[k] - e;
    const double CU = fma(w.cw, P, -(w.swq * s[k]));
    const double SU = fma(w.sw, P, w.cwq * s[k]);
    const double cu = CU * inv;
    const double su = SU * inv;
    const double b = inv;
    dd[k] = fma(CU, CU, w.ci2 * (SU * SU));  // sqrt only on eclipse lanes
    zz[k] = SU * w.si;
    const double b2 = b * b;
    // b^2 [A2 + b (A3 + b (A4 + b A5))] + kconst + kb cos u, the harmonics as
    // polynomials in x = sin^2 u (su2_form)
    const double x = su * su;
    const double a5 = fma(fma(w.kc4, x, w.kc22), x, w.kam3);
    const double a4 = su * fma(w.ks3, x, w.ks1);
    const double a3 = fma(w.kc21, x, w.kam2);
    const double a2 = fma(w.krs, su, fma(w.kr2, x, w.kr0));
    double h = fma(b, a5, a4);
    h = fma(b, h, a3);
    h = fma(b, h, a2);
    // values stay ~1 like the reference's Amag1 + Amag2 (one sign, one
    // exponent: the median radix-select resolves them in one digit pass)
    v[k] = fma(b2, h, fma(w.kb, cu, w.kconst));
  }
}
template <int K>
__device__ __forceinline__ void flux_poly_k(const double (&s)[K], const double (&c)[K], const WalkerConst& w,
                                            double (&v)[K], double (&dd)[K], double (&zz)[K]) {
  double inv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) inv[k] = fast_rcp(fma(-w.e, c[k], 1.0));
  flux_poly_inv_k<K>(s, c, inv, w, v, dd, zz);
}

// squared test: a lane within an ulp of tangency may go either way, where
// the overlap area (~eps^1.5) is zero to working precision
__device__ __forceinline__ bool eclipse_lane(const WalkerConst& w, double dd, double zz) {
  return (dd * w.aR2 < w.rsum2) & (zz != 0.0);
}

template <int K>
__device__ __forceinline__ void flux_from_sc_k(const double (&s)[K], const double (&c)[K], const WalkerConst& w,
                                               double (&v)[K]) {
  double dd[K], zz[K];
  flux_poly_k<K>(s, c, w, v, dd, zz);
  bool need_ecl = false;
#pragma unroll
  for (int k = 0; k < K; ++k) need_ecl |= eclipse_lane(w, dd[k], zz[k]);
  if (wave_any(need_ecl)) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (eclipse_lane(w, dd[k], zz[k])) v[k] -= eclipse_term(&w, sqrt(dd[k]) * w.aR, zz[k]);
    }
  }
}

// The asm barriers below split the walker constants' live ranges between the
// Kepler solve and the photometric polynomial: the constants are (re)loaded
// with scalar loads after the solve instead of being held in SGPRs across it,
// which would spill the solve's polynomial constants (SGPR spills 100 -> 52,
// no VGPR spills; eval 55.4 -> 54.1 us at C2, round 1).

// the polynomial part of K cadences, dd / zz for the caller's eclipse test
template <int K>
__device__ __forceinline__ void hb_cadence_poly_k(const double (&t)[K], const double2 (&ph)[K], bool tab,
                                                  const WalkerConst& w, double (&v)[K], double (&dd)[K],
                                                  double (&zz)[K], bool& bad) {
  double m[K], E[K], s[K], c[K], yk[K];
  bool ok = true, exact = false, plus[K];
  mean_anomaly_k<K>(t, w, m, plus, ok, exact);
  cold_start_k<K>(t, ph, tab, exact, w, m, plus, E, s, c, ok);
  (void)newton_k<K>(w.e, m, E, s, c, yk, ok);
  __asm__ volatile("" ::: "memory");
  flux_poly_k<K>(s, c, w, v, dd, zz);
  bad = !ok;
}

template <int K>
__device__ __forceinline__ void hb_cadence_flux_k(const double (&t)[K], const double2 (&ph)[K], bool tab,
                                                  const WalkerConst& w, double (&v)[K], bool& bad) {
  double m[K], E[K], s[K], c[K], yk[K];
  bool ok = true, exact = false, plus[K];
  mean_anomaly_k<K>(t, w, m, plus, ok, exact);
  cold_start_k<K>(t, ph, tab, exact, w, m, plus, E, s, c, ok);
  (void)newton_k<K>(w.e, m, E, s, c, yk, ok);
  __asm__ volatile("" ::: "memory");
  flux_from_sc_k<K>(s, c, w, v);
  bad = !ok;
}

// ------------------------------------------------------------------------
// Warm-started Kepler solve along a lane's consecutive cadences (the one-wave
// kernel, where lane l owns cadences l*VPT .. l*VPT + VPT - 1 as K chains).
// Consecutive cadences of a light curve are close in phase, so the previous
// cadence's root starts the next solve within O(dM^4) (third-order series
// reversion below): one Newton step instead of the reference start's three
// or four.  The root is the one the reference's five steps reach whenever
// those converge -- which holds for every M when e <= 0.85
// (scripts/kepler_warm.py) -- so the warm start is taken only for e <= 0.84
// (chain_eligible), and a lane outside the fast path continues with the
// general Newton loop, failing that from the reference's start
// (wave-uniform decisions throughout).
//
// A chain step comes in two halves, so the model pass can software-pipeline
// the chains (model_pass_chain_pipe, hb_kernels.hip): step j's Kepler solve
// and step j-1's photometric polynomial read the same chain state and are
// independent, so both sit in one basic block and interleave (twice the
// independent fp64 chains per lane: the drain, where one or two waves are left
// on a SIMD, is latency-bound).
// ------------------------------------------------------------------------
#ifndef HB_WARM_EMAX
#define HB_WARM_EMAX 0.84  // A/B knob (at most 0.85, see above; 0.8 until round 5: profiles/r05/r05za_warm_gate_ab.txt)
#endif
constexpr double kWarmEmax = HB_WARM_EMAX;
// The chain carries the previous cadence's solved E, (sin, cos)(E), its mean
// anomaly m and 1 / (1 - e cos E) (the polynomial's beta, which is also the
// warm start's 1 / f'(E_p)); the polynomial's reciprocal is seeded with the
// Newton step's 1 / f' (one ulp class from the final one: two Newton
// refinements make it full precision) instead of a fresh v_rcp_f64.
template <int K>
struct ChainState {
  double E[K], s[K], c[K];
  double inv[K];
  double m[K];  // the mean anomaly E solved: the next step's D = m' - m
};
// per-walker factors of the warm step, taken once per model pass
struct WarmK {
  double he, e6, ke;  // 0.5 e, e / 6, 2^-51 / e (the convergence test z <= ke den)
};
__device__ __forceinline__ WarmK warm_k(double e) { return WarmK{0.5 * e, e * (1.0 / 6.0), 0x1p-51 / fabs(e)}; }

// Warm half: the mean anomaly up to a multiple of 2pi (no exactness flags:
// D is reduced by rint), the third-order start -- series reversion of Kepler's
// equation about the previous root, E0 = E_p + x - A x^2 + (2 A^2 - B) x^3
// with x = dM / f1, A = f2 / (2 f1), B = f3 / (6 f1) at E_p (f1 = 1 - e cos,
// f2 = e sin, f3 = e cos), error O(x^4) -- then (sin, cos)(E0) by a degree-9
// rotation of the previous (sin, cos) and ONE Newton step.  fine: the lane's
// step is |d| <= 2^-22 with e d^2 <= 2^-51 (1 - e cos E), i.e. its next
// correction would be below 2^-52 (converged to rounding).
template <int K>
__device__ __forceinline__ void chain_kepler_warm(const double (&t)[K], const WalkerConst& w, const ChainState<K>& st,
                                                  double (&m)[K], double (&E)[K], double (&s)[K], double (&c)[K],
                                                  double (&ys)[K], bool& fine, bool& ok, const WarmK& wk) {
  const double e = w.e;
  const double he = wk.he, e6 = wk.e6;
  fine = true;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double x = fma(t[k], kDay, w.mB) * w.mA;
    ok &= sincos_fast_ok(x);
    m[k] = fma(-trunc(x * 0.15915494309189533577), kTwoPi, x);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double D = m[k] - st.m[k];
    const double q = rint(D * 0.15915494309189533577);
    const double Dc = fma(-q, kTwoPi, D);
    const double r = st.inv[k];
    const double x = Dc * r;
    const double A = (he * st.s[k]) * r;
    const double B = (e6 * st.c[k]) * r;
    const double C = fma(2.0 * A, A, -B);
    const double dl = fma(x * x, fma(C, x, -A), x);
    double E0 = fma(q, kTwoPi, st.E[k]) + dl;
    double s0 = st.s[k], c0 = st.c[k];
    const double z0 = dl * dl;
    fine &= fabs(dl) <= 0.0625;
    {  // rotate forward by dl: sin dl = dl (1 + z S(z)), cos dl = 1 + z C(z)
      const double sd = fma(dl * z0, fma(z0, fma(z0, fma(z0, 1.0 / 362880.0, -1.0 / 5040.0), 1.0 / 120.0),
                                         -1.0 / 6.0), dl);
      const double cd = fma(z0, fma(z0, fma(z0, fma(z0, 1.0 / 40320.0, -1.0 / 720.0), 1.0 / 24.0), -0.5), 1.0);
      const double s1 = fma(s0, cd, c0 * sd);
      const double c1 = fma(c0, cd, -(s0 * sd));
      s0 = s1;
      c0 = c1;
    }
    const double den = fma(-e, c0, 1.0);
    double y = __builtin_amdgcn_rcp(den);
    y = fma(fma(-den, y, 1.0), y, y);
    const double d = ((E0 - e * s0) - m[k]) * y;
    E0 = E0 - d;
    const double z = d * d;
    fine &= (fabs(d) <= 0x1p-22) & (z <= wk.ke * den);
    rotate_back_tiny(d, z, s0, c0);
    E[k] = E0;
    s[k] = s0;
    c[k] = c0;
    ys[k] = y;
  }
}
// the rest of a warm step once the wave knows whether every lane is fine:
// the reciprocal from the Newton step's seed, or the general Newton loop from
// the lane's iterate (a lane that was not fine first re-evaluates (sin, cos))
// and, failing that, the reference's start; then the chain state
template <int K>
__device__ __forceinline__ void chain_finish_warm(const double (&t)[K], const WalkerConst& w, bool all_fine,
                                                  bool fine, double (&m)[K], double (&E)[K], double (&s)[K],
                                                  double (&c)[K], const double (&ys)[K], bool& ok,
                                                  ChainState<K>& st) {
  const double e = w.e;
  if (all_fine) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double den = fma(-e, c[k], 1.0);
      double y = ys[k];
      y = fma(fma(-den, y, 1.0), y, y);
      st.inv[k] = fma(fma(-den, y, 1.0), y, y);
      st.E[k] = E[k];
      st.s[k] = s[k];
      st.c[k] = c[k];
      st.m[k] = m[k];
    }
    return;
  }
  if (!fine) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      ok &= sincos_fast_ok(E[k]);
      sincos_fast(E[k], &s[k], &c[k]);
    }
  }
  double yk[K];
  if (!newton_k<K>(e, m, E, s, c, yk, ok)) {  // redo from the reference's start
    bool plus[K], exact = false;
    ok = true;
    mean_anomaly_k<K>(t, w, m, plus, ok, exact);
    const double2 p0[K] = {};
    cold_start_k<K>(t, p0, false, exact, w, m, plus, E, s, c, ok);
    (void)newton_k<K>(e, m, E, s, c, yk, ok);
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    st.E[k] = E[k];
    st.s[k] = s[k];
    st.c[k] = c[k];
    st.inv[k] = fast_rcp(fma(-e, c[k], 1.0));
    st.m[k] = m[k];
  }
}
// a chain's first cadence: the reference's start (table entries) and Newton
template <int K>
__device__ __forceinline__ void chain_first(const double (&t)[K], const double2 (&ph)[K], bool tab, const WalkerConst& w,
                                            ChainState<K>& st, bool& ok) {
  const double e = w.e;
  double m[K], E[K], s[K], c[K], yk[K];
  bool exact = false, plus[K];
  mean_anomaly_k<K>(t, w, m, plus, ok, exact);
  cold_start_k<K>(t, ph, tab, exact, w, m, plus, E, s, c, ok);
  (void)newton_k<K>(e, m, E, s, c, yk, ok);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    st.E[k] = E[k];
    st.s[k] = s[k];
    st.c[k] = c[k];
    st.inv[k] = fast_rcp(fma(-e, c[k], 1.0));
    st.m[k] = m[k];
  }
}

}  // namespace hbdev
