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

template <int NW>
struct PrepShared {
  double sp[NW * kNpars];      // parameters of the group's walkers
  double so[NW * kWcDoubles];  // their records
  double xs[2][16][NW];        // per star: 0 m, 1 r, 2 tk, 3 ab, 4..15 star-2 terms
  double gs[3][NW];            // wave 2's Gaia term and sin/cos omega
};

struct PrepNoIdle {
  __device__ void operator()() const {}
};
// Records of the nb <= NW walkers whose parameters are in L.sp, into L.so.
// Every thread of the workgroup calls it (it holds two workgroup barriers and
// ends with a third).  tab/wt/base: catalog mode (the walker's target
// descriptor), else null.  tab_pc(j): the period [s] of the phase table walker
// j may use (NaN: no table).  slack(): wave 2's spare work after its own terms.
// Waves past the four roles (a workgroup of more than 256 threads: the fused
// eval kernel) run idle() between the first and the second barrier.
template <int NW, class TabPc, class Slack, class Idle = PrepNoIdle>
__device__ __forceinline__ void prep_records(PrepShared<NW>& L, int nb, const MagArgs& ma,
                                             const TargetDesc* __restrict__ tab, const int* __restrict__ wt,
                                             int base, TabPc tab_pc, Slack slack, Idle idle = Idle()) {
  static_assert(NW >= 1 && NW <= 64, "one walker per lane");
  const int tid = threadIdx.x;
  const int j = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform role
  if (wv >= kPrepRoles) {  // no role: the barriers, and the caller's work in between
    __syncthreads();
    idle();
    __syncthreads();
    __syncthreads();
    return;
  }
  const int star = wv & 1;
  const bool chainR = wv < 2;  // radius law + coefficients; else Teff law + tail
  const bool live = j < nb;
  const int jc = live ? j : 0;
  const double* p = &L.sp[jc * kNpars];

  // ---- this wave's half of the star (calc_radii_and_Teffs + get_alpha_beam) ----
  const double m = exp10(p[star]);
  if (chainR) {
    const double r = exp10(logradius_of_mass(m) + p[7 + star] * radius_spread_of_logmass(p[star]));
    if (live) {
      L.xs[star][0][j] = m;
      L.xs[star][1][j] = r;
    }
  } else {
    const double lt = logteff_of_mass(m) + p[17 + star] * teff_spread();
    const double tk = exp10(lt);
    const double ab = beam_coeff(lt) * exp(p[15 + star]);
    if (live) {
      L.xs[star][2][j] = tk;
      L.xs[star][3][j] = ab;
    }
  }
  const double pd = exp10(p[2]);
  const double e = p[3];
  HB_PREP_MARK(5 + wv);  // phase 1 computed (values in registers / LDS stores issued)
  __syncthreads();
  const int o = star ^ 1;
  const double r = L.xs[star][1][jc], tk = L.xs[star][2][jc], ab = L.xs[star][3][jc];
  const double mo = L.xs[o][0][jc], ro = L.xs[o][1][jc], tko = L.xs[o][2][jc];
  const double lum = sq(r) * sq(sq(tk));
  const double lumo = sq(ro) * sq(sq(tko));
  // the same sum in every wave: star-1 luminosity first
  const double lsum = star ? (lumo + lum) : (lum + lumo);
  const double m1 = star ? mo : m, m2 = star ? m : mo;
  const double r1 = star ? ro : r, r2 = star ? r : ro;
  const double t1 = star ? tko : tk, t2 = star ? tk : tko;
  WalkerConst* wc = reinterpret_cast<WalkerConst*>(&L.so[jc * kWcDoubles]);
  double si = 0.0, ci = 0.0;
  double aR = 0.0, sq1me2 = 0.0, inv1me2 = 0.0, mA = 0.0;  // wave 0's orbit fields, off the last phase
  if (chainR) {
    sincos(p[4], &si, &ci);
    if (star == 0) {
      const double mtot_cgs = m1 * kMsun + m2 * kMsun;
      const double Pc = pd * kDay;
      aR = cbrt(kG * mtot_cgs * (Pc * Pc) / (kTwoPi * kTwoPi)) / kRsun;
      sq1me2 = sqrt(1.0 - e * e);
      inv1me2 = 1.0 / (1.0 - e * e);
      mA = kTwoPi / Pc;
    }
    const double nself = lum / lsum;
    const StarCoef c = star_coef(pd, m, mo, e, si, r, ro, p[9 + 2 * star], p[10 + 2 * star], p[13 + star], ab);
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
    if (live) {  // both stars' terms through LDS (no 12 registers held across the barrier)
#pragma unroll
      for (int q = 0; q < 12; ++q) L.xs[star][4 + q][j] = terms[q];
    }
  } else if (star == 1) {
    if (live) {
      const double mtot_cgs = m1 * kMsun + m2 * kMsun;
      const double Pc = pd * kDay;
      const double a_cgs = cbrt(kG * mtot_cgs * (Pc * Pc) / (kTwoPi * kTwoPi));
      // eclipse geometry
      wc->r1 = r1;
      wc->r2 = r2;
      const double lum1 = star ? lumo : lum, lum2 = star ? lum : lumo;
      const double n1 = lum1 / lsum, n2 = lum2 / lsum;
      wc->ecl1 = n1 / (kPi * (r1 * r1));
      wc->ecl2 = n2 / (kPi * (r2 * r2));
      wc->rbig = r2 > r1 ? r2 : r1;
      wc->rsml = r2 > r1 ? r1 : r2;
      wc->dcrit = sqrt(wc->rbig * wc->rbig - wc->rsml * wc->rsml);
      wc->rsum = wc->rbig + wc->rsml;
      wc->rsum2 = wc->rsum * wc->rsum;
      // Roche overflow (RocheOverflow :953-974)
      const double q12 = m1 / m2;
      const double peri = a_cgs * (1.0 - e);
      const double f1 = (r1 * kRsun) / peri;
      const double f2 = (r2 * kRsun) / peri;
      wc->roche = ((lobe_fraction(q12) < f1) || (lobe_fraction(1.0 / q12) < f2)) ? 1.0 : 0.0;
      // phase-table rotations (WalkerConst::tab); same Pc and mA as wave 0's orbit fields
      const bool use_tab = Pc == tab_pc(j);  // false for NaN (no table)
      wc->tab = use_tab ? 1.0 : 0.0;
      double sv = 0.0, cv = 1.0;
      if (use_tab) sincos_table((p[6] * kDay) * (kTwoPi / Pc), sv, cv);
      wc->spsi = sv;
      wc->cpsi = cv;
      sincos_table(0.85 * e, sv, cv);
      wc->sdel = sv;
      wc->cdel = cv;
      wc->pad0 = 0.0;
    }
  } else {
    // Gaia G term (loglikelihood :834-848)
    double dist = ma.mag[0], gobs = ma.mag[1], gerr = ma.magerr[0];
    if (tab != nullptr && live) {  // catalog mode: this walker's target
      const TargetDesc& td = tab[wt[base + j]];
      dist = td.dist;
      gobs = td.gmag;
      gerr = td.gerr;
    }
    const double g = ab_mag(band_flux(673.0, r1 * kRsun, r2 * kRsun, t1, t2, dist, p[19]));
    double sw_, cw_;
    sincos(p[5], &sw_, &cw_);
    if (live) {
      L.gs[0][j] = (g - gobs) / gerr;
      L.gs[1][j] = sw_;
      L.gs[2][j] = cw_;
    }
    slack();
  }
  HB_PREP_MARK(9 + wv);  // phase 2 computed
  __syncthreads();  // star-2 terms and the Gaia term are in LDS
  if (wv == 0 && live) {
    double tt[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) tt[q] = L.xs[0][4 + q][j] + L.xs[1][4 + q][j];  // star-1 term first
    const double gr = L.gs[0][j];
    // orbit
    wc->Pc = pd * kDay;
    wc->T0c = p[6] * kDay;
    wc->e = e;
    wc->e085 = 0.85 * e;
    wc->sq1me2 = sq1me2;
    wc->inv1me2 = inv1me2;
    wc->sw = L.gs[1][j];
    wc->cw = L.gs[2][j];
    wc->ci = ci;
    wc->si = si;
    wc->ci2 = ci * ci;
    wc->swq = L.gs[1][j] * sq1me2;
    wc->cwq = L.gs[2][j] * sq1me2;
    wc->aR = aR;
    wc->aR2 = aR * aR;
    wc->mA = mA;
    wc->mB = -wc->T0c;
    // polynomial coefficients
    const double s2 = si * si;
    wc->kconst = tt[11] + tt[0];
    wc->kb = tt[1];
    wc->kr0 = tt[2] * (0.64 + 0.18 * s2);
    wc->kr2 = -tt[2] * (0.18 * s2);
    wc->krs = -tt[3] * si;
    wc->kam2 = tt[4];
    wc->kc21 = tt[5];
    wc->ks1 = tt[6];
    wc->ks3 = tt[7];
    wc->kam3 = tt[8];
    wc->kc22 = tt[9];
    wc->kc4 = tt[10];
    wc->blend = p[19];
    wc->tune = p[20];
    wc->chi2_extra = gr * gr;
  }
  HB_PREP_MARK(13);  // wave 0: records combined (other waves: no-op)
  __syncthreads();
}

}  // namespace hbk
