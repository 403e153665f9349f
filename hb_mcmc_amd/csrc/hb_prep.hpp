// hb_prep.hpp -- per-walker constants (WalkerConst, hb_device.hpp) from the 21
// parameters: calc_radii_and_Teffs, get_alpha_beam, the light-curve
// coefficients, eclipse geometry, RocheOverflow and the Gaia term
// (likelihood3.c:533-648, 725-795, 834-848, 945-974).
//
// One prep group = four waves with wave-uniform roles and one walker per lane
// (NW <= 64 walkers): wave s (s = star 0/1) runs the star's radius law and
// then its photometric coefficients; wave 2 + s runs the star's Teff law and
// beaming factor, then a star-specific tail (wave 2: Gaia term and sin/cos
// omega, plus the caller's spare work; wave 3: eclipse geometry, Roche test and
// phase-table rotations).  The group is latency-bound, so splitting the
// independent chains over four waves shortens the critical path; results cross
// waves through LDS.  Used by
//   hb_prep_kernel (hb_kernels.hip): the batched API, NW = kPrepWalkers walkers
//       per workgroup, parameters and records moved through LDS so the HBM
//       accesses coalesce;
//   ds_propose (hb_dsampler.hip): the device sampler, whose workgroup of four
//       proposal waves (one slot each) turns into one prep group of NW = 4 in
//       its epilogue -- no separate launch per iteration.
// Both run the same operations in the same order: bit-identical records.
#pragma once
#include <hip/hip_runtime.h>

#include "hb_device.hpp"
#include "hb_internal.hpp"

// experiment builds only (HB_WAVE_CLOCKS, hb_kernels.hip): shader-clock marks
// of the prep roles, mark i of the calling wave's lane 0
#ifndef HB_PREP_MARK
#define HB_PREP_MARK(i) do { } while (0)
#endif

namespace hbk {

using namespace hbdev;

constexpr int kWcDoubles = (int)(sizeof(WalkerConst) / sizeof(double));
constexpr int kPrepRoles = 4;  // waves per prep group

// sin/cos of a phase-table angle: the branch-free reduction for |x| < 2^19,
// ocml otherwise (never for folded light curves)
__device__ __forceinline__ void sincos_table(double x, double& sv, double& cv) {
  if (sincos_fast_ok(x)) {
    sincos_fast(x, &sv, &cv);
  } else {
    const SinCos r = sincos_ocml(x);
    sv = r.s;
    cv = r.c;
  }
}

// A walker's record in LDS takes kSoStride doubles: an odd stride, so the
// lanes' record stores and loads (lane = walker) hit distinct banks (a stride
// of 48 doubles put 16 lanes on 2 banks)
constexpr int kSoStride = kWcDoubles + 1;

template <int NW>
struct PrepShared {
  double sp[NW * kNpars];      // parameters of the group's walkers
  double so[NW * kSoStride];   // their records (row stride kSoStride)
  // per star: 0 Planck factor (Gaia band), 1 r, 2 tk, 3 ab; 4..15 the radius-free
  // coefficient factors (StarCoefX, phase 1), then the star's terms (phase 2)
  double xs[2][16][NW];
  double gs[4][NW];            // Gaia term, periastron [cm], Roche-lobe fractions of star 1 and 2
};

struct PrepNoIdle {
  __device__ void operator()() const {}
};

// Lane tasks.  Waves 0-2 run per-star chains with lane k = star * NW + walker
// (k < 2 NW; NW = 64 takes two passes): both stars' chains are the same
// instruction stream, so one wave does both for the issue cost of one.  Wave
// 3's lane k = half * NW + walker runs the walker's orbit and pairs of
// like computations (sin/cos of i and omega, the two Roche lobes, the two
// phase-table rotations), one of each pair per half.
template <int NW>
struct PrepTask {
  int star, j, jc;
  bool live;
  __device__ PrepTask(int k, int nb) {
    star = k >= NW ? 1 : 0;
    j = k - star * NW;
    live = k < 2 * NW && j < nb;
    jc = live ? j : 0;
  }
};

// The light-curve polynomial's coefficients from both stars' summed terms
// tt (star 1's term first) and sin i (already in the record)
__device__ __forceinline__ void prep_coefficients(double* rec, WalkerConst* wc, const double (&tt)[12]) {
#define HB_REC(field) rec[&wc->field - (double*)wc]
  const double si = HB_REC(si);
  const double s2 = si * si;
  HB_REC(kconst) = tt[11] + tt[0];
  HB_REC(kb) = tt[1];
  HB_REC(kr0) = tt[2] * (0.64 + 0.18 * s2);
  HB_REC(kr2) = -tt[2] * (0.18 * s2);
  HB_REC(krs) = -tt[3] * si;
  HB_REC(kam2) = tt[4];
  HB_REC(kc21) = tt[5];
  HB_REC(ks1) = tt[6];
  HB_REC(ks3) = tt[7];
  HB_REC(kam3) = tt[8];
  HB_REC(kc22) = tt[9];
  HB_REC(kc4) = tt[10];
  su2_form(HB_REC(kr0), HB_REC(kr2), HB_REC(kam2), HB_REC(kc21), HB_REC(ks1), HB_REC(ks3), HB_REC(kam3), HB_REC(kc22),
           HB_REC(kc4));
#undef HB_REC
}

// Records of the nb <= NW walkers whose parameters are in L.sp, into L.so
// (row j at L.so[j * kSoStride]).  Every thread of the workgroup calls it (it
// holds one workgroup barrier -- two when NW = 64 -- and ends with another).  tab/wt/base: catalog
// mode (the walker's target descriptor), else null.  tab_pc(j): the period
// [s] of the phase table walker j may use (NaN: no table).  slack(): wave 2's
// spare work (phase 2).  Waves past the four roles (a workgroup of more than
// 256 threads: the fused eval kernel) run idle() before the first barrier.
//
// Phase 1 (before the first barrier) holds every chain that needs no other
// wave's result, split so that no wave carries much more issue than another:
//   wave 0: the radius law and the Roche-lobe fraction (both stars);
//   wave 1: each star's coefficient factors that need no radius (star_coef_x,
//           with its own sin i);
//   wave 2: the Teff law, alpha_beam and the Gaia-band Planck factor;
//   wave 3: the orbit fields, sin/cos i | omega, periastron and
//           the phase-table rotations, straight into the record.
// Phase 2 only combines values across waves: wave 1 multiplies the radii in
// (star_coef_r, star_coef_finish), weights each star's terms and sums the two
// stars' into the polynomial coefficients (lane shuffles; with two passes,
// NW = 64, through LDS after another barrier); wave 3 the eclipse geometry
// and Roche test; wave 0 the Gaia term; wave 2 runs slack().
template <int NW, class TabPc, class Slack, class Idle = PrepNoIdle>
__device__ __forceinline__ void prep_records(PrepShared<NW>& L, int nb, const MagArgs& ma,
                                             const TargetDesc* __restrict__ tab, const int* __restrict__ wt,
                                             int base, TabPc tab_pc, Slack slack, Idle idle = Idle()) {
  static_assert(NW >= 1 && NW <= 64, "one walker per lane");
  constexpr int kPass = (2 * NW + 63) / 64;
  // one pass (NW <= 32): both stars' terms meet by lane shuffles in phase 2
  // (two barriers in all); two passes: through LDS after a third barrier
  constexpr bool kShfl = kPass == 1;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform role
  if (wv >= kPrepRoles) {  // no role: the caller's work, then the barriers
    idle();
    __syncthreads();
    __syncthreads();
    if (!kShfl) __syncthreads();
    return;
  }
  // ---- phase 1 ----
  if (wv == 0) {  // radius law
#pragma unroll
    for (int ps = 0; ps < kPass; ++ps) {
      const PrepTask<NW> k(lane + 64 * ps, nb);
      const double* p = &L.sp[k.jc * kNpars];
      const double m = exp10(p[k.star]);
      const double r = exp10(logradius_of_mass(m) + p[7 + k.star] * radius_spread_of_logmass(p[k.star]));
      // the star's Roche-lobe fraction (RocheOverflow :953-974: q12 = M1/M2, star 2 at 1/q12)
      const double mo = exp10(p[k.star ^ 1]);
      const double q12 = k.star ? mo / m : m / mo;
      const double lf = lobe_fraction(k.star ? 1.0 / q12 : q12);
      if (k.live) {
        L.xs[k.star][1][k.j] = r;
        L.gs[2 + k.star][k.j] = lf;
      }
    }
  } else if (wv == 1) {  // radius-free coefficient factors
#pragma unroll
    for (int ps = 0; ps < kPass; ++ps) {
      const PrepTask<NW> k(lane + 64 * ps, nb);
      const double* p = &L.sp[k.jc * kNpars];
      const double pd = exp10(p[2]);
      const double m = exp10(p[k.star]);
      const double mo = exp10(p[k.star ^ 1]);
      double si, ci;
      sincos(p[4], &si, &ci);
      const StarCoefX x = star_coef_x(pd, m, mo, p[3], si, p[9 + 2 * k.star], p[10 + 2 * k.star], p[13 + k.star]);
      if (k.live) {
        double* d = &L.xs[k.star][4][k.j];
        d[0 * NW] = x.kb;
        d[1 * NW] = x.am1;
        d[2 * NW] = x.am2;
        d[3 * NW] = x.c21;
        d[4 * NW] = x.a3;
        d[5 * NW] = x.a22;
        d[6 * NW] = x.a4;
        d[7 * NW] = x.x5;
        d[8 * NW] = x.b1;
        d[9 * NW] = x.b3;
        d[10 * NW] = x.x4;
        d[11 * NW] = x.kref;
      }
    }
  } else if (wv == 2) {  // Teff law, alpha_beam, Gaia-band Planck factor
#pragma unroll
    for (int ps = 0; ps < kPass; ++ps) {
      const PrepTask<NW> k(lane + 64 * ps, nb);
      const double* p = &L.sp[k.jc * kNpars];
      const double m = exp10(p[k.star]);
      const double lt = logteff_of_mass(m) + p[17 + k.star] * teff_spread();
      const double tk = exp10(lt);
      const double ab = beam_coeff(lt) * exp(p[15 + k.star]);
      const double bt = band_term(673.0, tk);
      if (k.live) {
        L.xs[k.star][0][k.j] = bt;
        L.xs[k.star][2][k.j] = tk;
        L.xs[k.star][3][k.j] = ab;
      }
    }
  } else {  // orbit, pairs (half = k.star)
#pragma unroll
    for (int ps = 0; ps < kPass; ++ps) {
      const PrepTask<NW> k(lane + 64 * ps, nb);
      const bool h1 = k.star != 0;
      const double* p = &L.sp[k.jc * kNpars];
      const double pd = exp10(p[2]);
      const double e = p[3];
      const double m1 = exp10(p[0]);
      const double m2 = exp10(p[1]);
      const double mtot_cgs = m1 * kMsun + m2 * kMsun;
      const double Pc = pd * kDay;
      const double a_cgs = cbrt(kG * mtot_cgs * (Pc * Pc) / (kTwoPi * kTwoPi));
      const double sq1me2 = sqrt_1me2(e);  // NaN at |e| >= 1 (hb_device.hpp)
      double sa, ca;  // (sin, cos) of i (half 0) or omega (half 1)
      sincos(h1 ? p[5] : p[4], &sa, &ca);
      // phase-table rotations: psi = T0 2pi/P (half 0, walkers on the table
      // period), del = 0.85 e (half 1)
      const bool use_tab = h1 || Pc == tab_pc(k.jc);  // false for NaN (no table)
      double sv, cv;
      sincos_table(h1 ? 0.85 * e : (p[6] * kDay) * (kTwoPi / Pc), sv, cv);
      if (!use_tab) {
        sv = 0.0;
        cv = 1.0;
      }
      if (k.live) {
        double* rec = &L.so[k.j * kSoStride];
        WalkerConst* wc = reinterpret_cast<WalkerConst*>(rec);  // field offsets only (odd row stride)
#define HB_REC(field) rec[&wc->field - (double*)wc]
        if (!h1) {
          const double T0c = p[6] * kDay;
          const double aR = a_cgs / kRsun;
          HB_REC(Pc) = Pc;
          HB_REC(T0c) = T0c;
          HB_REC(e) = e;
          HB_REC(e085) = 0.85 * e;
          HB_REC(sq1me2) = sq1me2;
          HB_REC(inv1me2) = 1.0 / (1.0 - e * e);
          HB_REC(si) = sa;
          HB_REC(ci) = ca;
          HB_REC(ci2) = ca * ca;
          HB_REC(aR) = aR;
          HB_REC(aR2) = aR * aR;
          HB_REC(mA) = kTwoPi / Pc;
          HB_REC(mB) = -T0c;
          HB_REC(tab) = use_tab ? 1.0 : 0.0;
          HB_REC(spsi) = sv;
          HB_REC(cpsi) = cv;
          HB_REC(pad0) = 0.0;
          L.gs[1][k.j] = a_cgs * (1.0 - e);  // periastron
        } else {
          HB_REC(sw) = sa;
          HB_REC(cw) = ca;
          HB_REC(swq) = sa * sq1me2;
          HB_REC(cwq) = ca * sq1me2;
          HB_REC(sdel) = sv;
          HB_REC(cdel) = cv;
        }
      }
    }
  }
  HB_PREP_MARK(5 + wv);  // phase 1 computed
  __syncthreads();
  // ---- phase 2: across the waves ----
  if (wv == 1) {  // the radii into each star's coefficients, weighted by its luminosity share
#pragma unroll
    for (int ps = 0; ps < kPass; ++ps) {
      const PrepTask<NW> k(lane + 64 * ps, nb);
      const int jc = k.jc, star = k.star;
      const double r1 = L.xs[0][1][jc], r2 = L.xs[1][1][jc];
      const double t1 = L.xs[0][2][jc], t2 = L.xs[1][2][jc];
      const double lum1 = sq(r1) * sq(sq(t1)), lum2 = sq(r2) * sq(sq(t2));
      const double lsum = lum1 + lum2;  // star-1 luminosity first
      double* d = &L.xs[star][4][jc];
      StarCoefX x;
      x.kb = d[0 * NW];
      x.am1 = d[1 * NW];
      x.am2 = d[2 * NW];
      x.c21 = d[3 * NW];
      x.a3 = d[4 * NW];
      x.a22 = d[5 * NW];
      x.a4 = d[6 * NW];
      x.x5 = d[7 * NW];
      x.b1 = d[8 * NW];
      x.b3 = d[9 * NW];
      x.x4 = d[10 * NW];
      x.kref = d[11 * NW];
      StarCoef c = star_coef_r(x, star ? r2 : r1);
      star_coef_finish(c, star ? r1 : r2, L.xs[star][3][jc]);
      const double nself = (star ? lum2 : lum1) / lsum;
      // star 2 sees u + pi: odd harmonics flip sign
      const double sg = star ? -1.0 : 1.0;
      double terms[12];
      terms[0] = nself * c.am1;
      terms[1] = nself * c.kb * sg;
      terms[2] = nself * c.kref;
      terms[3] = sg * nself * c.kref;
      terms[4] = nself * c.am2;
      terms[5] = nself * c.c21;
      terms[6] = sg * nself * c.s1;
      terms[7] = sg * nself * c.s3;
      terms[8] = nself * c.am3;
      terms[9] = nself * c.c22;
      terms[10] = nself * c.c4;
      terms[11] = nself;
      if constexpr (kShfl) {
        // star 2's terms from lane j + NW; lane j (star 1) sums them into the
        // walker's coefficients (star-1 term first, like the LDS path below)
        double o[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) o[q] = __shfl(terms[q], lane + NW, 64);
        if (star == 0 && k.live) {
          double tt[12];
#pragma unroll
          for (int q = 0; q < 12; ++q) tt[q] = terms[q] + o[q];
          double* rec = &L.so[k.j * kSoStride];
          WalkerConst* wc = reinterpret_cast<WalkerConst*>(rec);
          prep_coefficients(rec, wc, tt);
        }
      } else if (k.live) {  // over the factors just read (same lane)
#pragma unroll
        for (int q = 0; q < 12; ++q) d[q * NW] = terms[q];
      }
    }
  } else if (wv == 3) {  // eclipse geometry, Roche test
    const int j = lane;
    const bool live = j < nb;
    const int jc = live ? j : 0;
    const double r1 = L.xs[0][1][jc], r2 = L.xs[1][1][jc];
    const double t1 = L.xs[0][2][jc], t2 = L.xs[1][2][jc];
    const double lum1 = sq(r1) * sq(sq(t1)), lum2 = sq(r2) * sq(sq(t2));
    const double lsum = lum1 + lum2;
    if (live) {
      double* rec = &L.so[j * kSoStride];
      WalkerConst* wc = reinterpret_cast<WalkerConst*>(rec);
      HB_REC(r1) = r1;
      HB_REC(r2) = r2;
      const double n1 = lum1 / lsum, n2 = lum2 / lsum;
      HB_REC(ecl1) = n1 / (kPi * (r1 * r1));
      HB_REC(ecl2) = n2 / (kPi * (r2 * r2));
      const double rbig = r2 > r1 ? r2 : r1, rsml = r2 > r1 ? r1 : r2;
      HB_REC(rbig) = rbig;
      HB_REC(rsml) = rsml;
      HB_REC(dcrit) = sqrt(rbig * rbig - rsml * rsml);
      const double rsum = rbig + rsml;
      HB_REC(rsum) = rsum;
      HB_REC(rsum2) = rsum * rsum;
      // Roche overflow (RocheOverflow :953-974)
      const double peri = L.gs[1][j];
      const double f1 = (r1 * kRsun) / peri;
      const double f2 = (r2 * kRsun) / peri;
      HB_REC(roche) = ((L.gs[2][j] < f1) || (L.gs[3][j] < f2)) ? 1.0 : 0.0;
    }
  } else if (wv == 0) {  // Gaia G term (loglikelihood :834-848)
    const int j = lane;
    const bool live = j < nb;
    const int jc = live ? j : 0;
    double dist = ma.mag[0], gobs = ma.mag[1], gerr = ma.magerr[0];
    if (tab != nullptr && live) {  // catalog mode: this walker's target
      const TargetDesc& td = tab[wt[base + j]];
      dist = td.dist;
      gobs = td.gmag;
      gerr = td.gerr;
    }
    const double r1 = L.xs[0][1][jc], r2 = L.xs[1][1][jc];
    const double g = ab_mag(band_flux_terms(r1 * kRsun, r2 * kRsun, L.xs[0][0][jc], L.xs[1][0][jc], dist,
                                            L.sp[jc * kNpars + 19]));
    if (live) {
      const double gr = (g - gobs) / gerr;
      double* rec = &L.so[j * kSoStride];
      WalkerConst* wc = reinterpret_cast<WalkerConst*>(rec);
      HB_REC(blend) = L.sp[j * kNpars + 19];
      HB_REC(tune) = L.sp[j * kNpars + 20];
      HB_REC(chi2_extra) = gr * gr;
    }
  } else {
    slack();
  }
  HB_PREP_MARK(9 + wv);  // phase 2 computed
  __syncthreads();  // two passes: both stars' terms are in LDS
  if constexpr (!kShfl) {
    if (wv == 0 && lane < nb) {
      const int j = lane;
      double tt[12];
#pragma unroll
      for (int q = 0; q < 12; ++q) tt[q] = L.xs[0][4 + q][j] + L.xs[1][4 + q][j];  // star-1 term first
      double* rec = &L.so[j * kSoStride];
      prep_coefficients(rec, reinterpret_cast<WalkerConst*>(rec), tt);
    }
    __syncthreads();
  }
#undef HB_REC
}

}  // namespace hbk
