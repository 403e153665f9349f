// hb_host.cpp -- host-side configuration tables of the likelihood3.h ABI.
// set_limits (likelihood3.c:986-1121) and initialize_proposals
// (likelihood3.c:1123-1211) only fill constant tables (prior box, Gaussian
// prior flags, proposal widths); there is no arithmetic to offload.
#include "../../include/hbmi.h"

namespace {
// {limited.lo, lo, limited.hi, hi, gauss flag} per slot, in slot order.
// NB limited[3].hi is 0.99 in the reference (not 1): e has no upper wall.
struct Slot {
  double lim_lo, lo, lim_hi, hi;
  int gauss;
};
const double kPI = 3.14159265358979323846;
}  // namespace

extern "C" void set_limits(bounds limited[], bounds limits[], gauss_bounds gauss_pars[], double LC_PERIOD) {
  const Slot tab[HBMI_NPARS] = {
      {1, -1.5, 1, 2.0, 0},        // 0 log M1 [log Msun]
      {1, -1.5, 1, 2.0, 0},        // 1 log M2
      {1, -2.0, 1, 3.0, 0},        // 2 log P [log d]
      {1, 0.0, 0.99, 1, 0},        // 3 e
      {1, 0, 1, kPI, 0},           // 4 inc [rad]
      {2, -kPI, 2, kPI, 0},        // 5 omega0 (periodic)
      {1, 0., 1, LC_PERIOD, 0},    // 6 T0 [d]
      {1, -5., 1, 5., 1},          // 7 rr1
      {1, -5., 1, 5., 1},          // 8 rr2
      {1, 0.12, 1, 0.20, 1},       // 9 mu1
      {1, 0.3, 1, 0.38, 1},        // 10 tau1
      {1, 0.12, 1, 0.20, 1},       // 11 mu2
      {1, 0.3, 1, 0.38, 1},        // 12 tau2
      {1, 0.5, 1, 1.5, 1},         // 13 alpha_ref1
      {1, 0.5, 1, 1.5, 1},         // 14 alpha_ref2
      {1, -0.3, 1, 0.3, 1},        // 15 ln beam1
      {1, -0.3, 1, 0.3, 1},        // 16 ln beam2
      {1, -5., 1, 5., 1},          // 17 alpha_Teff1
      {1, -5., 1, 5., 1},          // 18 alpha_Teff2
      {1, 0., 1, 1., 0},           // 19 blending
      {1, 0.99, 1, 1.01, 0},       // 20 flux_tune
  };
  for (int i = 0; i < HBMI_NPARS; ++i) {
    limited[i].lo = tab[i].lim_lo;
    limits[i].lo = tab[i].lo;
    limited[i].hi = tab[i].lim_hi;
    limits[i].hi = tab[i].hi;
    gauss_pars[i].flag = tab[i].gauss;
  }
}

// Proposal widths after the "no colour info" override (likelihood3.c:1157-1179,
// which always fires with USE_COLOR_INFO=0).  `history` is not touched (its
// reader is commented out in the reference, :1195-1210).
extern "C" void initialize_proposals(double* sigma, double*** history) {
  (void)history;
  const double s[HBMI_NPARS] = {1.e-1, 1.e-1, 1.0e-8, 1.0e-2, 1.e-2, 1.e-2, 1.e-3,
                                1.0e-1, 1.0e-1, 1.e-1, 1.e-1, 1.e-1, 1.e-1, 1.e-1,
                                1.e-1, 1.e-1, 1.e-1, 1.e-1, 1.e-1, 1.0e-3, 1.0e-5};
  for (int i = 0; i < HBMI_NPARS; ++i) sigma[i] = s[i];
}
