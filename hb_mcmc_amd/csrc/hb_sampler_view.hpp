// hb_sampler_view.hpp -- internal bridge between the host sampler
// (hb_sampler.cpp, g++) and the device-resident sampler (hb_dsampler.hip):
// plain pointers into a hb_sampler's state, so a device run can start from a
// host sampler and hand the exact state back.  Not part of the public ABI.
#pragma once
#include <stdint.h>
#include "../../include/hb_sampler.h"
#include "../../include/hbmi.h"

struct HbSamplerView {
  int W, NPAST, lo, hi, nl;
  long NITER;
  double log_lc_period, LC_PERIOD;
  const bounds* limited;     // [21] wall flags (1 reflecting, 2 periodic)
  const bounds* limits;      // [21]
  const gauss_bounds* gp;    // [21] prior flags
  const double* sigma_p;     // [21] proposal widths
  const double* temp;        // [W]  ladder
  long* seeds;               // [nl] ran2 idum
  RNG_Vars* states;          // [nl]
  double* x;                 // [nl x 21] by slot
  double* logL;              // [nl]
  double* logP;              // [nl]
  char* logP_ok;             // [nl]
  int* cid;                  // [nl] chain id at the slot
  double* hist;              // [nl x NPAST x 21]
  int* acc_arr;              // [nl]
  int* DEacc_arr;            // [nl]
  int* DEtrial_arr;          // [nl]
  long* acc;                 // scalar counters
  long* DEacc;
  long* DEtrial;
  long* atrial;
  long* cold_acc;
  long* nswap;
  hb_writer* log;            // big-jump log (may be NULL)
};

extern "C" {
int hbx_sampler_view(hb_sampler* s, HbSamplerView* v);
// the next 2W glibc rand() draws of the sampler's swap stream, as the
// reference's ptmcmc consumes them (mcmc_wrapper2.c:791, :810): per attempt
// i, b[i] = (int)(rand()/RAND_MAX * (W-1)) and beta[i] = rand()/RAND_MAX
int hbx_swap_draws(hb_sampler* s, int* b, double* beta);
// the swap stream's state as the window of its last 31 outputs
// (hb_lagfib.hpp), and a jump-ahead of n draws
int hbx_swap_rng_window(const hb_sampler* s, uint32_t* w31);
int hbx_swap_rng_skip(hb_sampler* s, unsigned long long n);
void hbx_log_big_jump(hb_writer* w, long iter, int chain_id, double H, double alpha, double tmp, double lx,
                      double ly, double px, double py, const double* xo, const double* xn, int jump_type);
}
