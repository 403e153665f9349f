// hb_dsampler.hip -- the PT-MCMC step of mcmc_wrapper2.c (:378-650) resident
// on the GPU: proposals, walls, priors, likelihood, Hastings test, history and
// the tempering swaps all run as kernels on one stream, so an iteration never
// waits for the host.  Results are bit-identical to the host sampler
// (hb_sampler.cpp) and so to the reference's bookkeeping:
//   * the integer L'Ecuyer/Bays-Durham streams (ran2_parallel :894-943) run
//     per slot in 32-bit arithmetic (Schrage's products stay below 2^31), the
//     shuffle table staged in LDS;
//   * every libm call on the state path goes through hb_glibc_math.hpp, the
//     bit-exact port of the host glibc's exp/log/pow; sqrt and division are
//     IEEE (correctly rounded) on gfx950 as on x86;
//   * the W sequential ptmcmc attempts (:768-817) consume glibc rand() in a
//     fixed order that does not depend on the data, so the host draws them
//     ahead (hbx_swap_draws) and sorts the attempts into dependency levels:
//     attempt i touches slots b_i, b_i + 1 and must follow every earlier
//     attempt that touches either; attempts within a level touch disjoint
//     slots and commute.  One workgroup then replays the ~10 levels (W = 4096)
//     with the exact exp() test, index[] and logL in LDS.
// State is kept by chain id like the reference (x[chain], logL[chain],
// index[slot] -> chain), so a swap moves one int, not a 23-double record.
//
// Sharded (one rank of R): the rank owns the contiguous slots
// [lo, lo + nl), lo = W r / R, with their RNG streams, proposals and history
// (arrays "by slot" hold only those, local index j - lo).  index[] and the
// arrays by chain keep all W entries; a chain's record is valid where its
// slot is owned.  Per iteration the rank proposes, evaluates and tests its
// slots, then ONE all-gather (the caller's collective, RCCL) carries
//   * logL of every owned slot (the tempering swaps need all W), and
//   * the records {chain, logP, logP_ok, x[21]} of the chains in the slots
//     within nlv of the shard's edges: a swap level moves a chain by at most
//     one slot, so with nlv levels only those chains can leave the shard;
// every rank then replays the identical swap schedule (same glibc stream,
// same logL) on its copy of index[] after importing the other ranks' records,
// so all ranks hold the same index[] and every owned slot's chain record.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <math.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hb_sampler.h"
#include "../../include/hbmi.h"
#include "hb_accept.hpp"
#include "hb_glibc_math.hpp"
#include "hb_lagfib.hpp"
#include "hb_prep.hpp"
#include "hb_sampler_view.hpp"
#include "hb_walls.hpp"
#include "hb_wave.hpp"

extern "C" int hbx_set_error(const char* msg);
extern "C" int hbx_ctx_device(const hb_ctx* c);
extern "C" int hbx_ctx_prep_args(hb_ctx* c, void** wc, void* mags, double** tab_pc);
extern "C" int hbx_loglik_accept_dev(hb_ctx* c, const double* d_params, int w, double* d_logl, const void* acc,
                                     void* stream);

namespace hbds {

constexpr int NTAB = 32;
constexpr int IM1 = 2147483563, IM2 = 2147483399, IMM1 = IM1 - 1;
constexpr int IA1 = 40014, IA2 = 40692, IQ1 = 53668, IR1 = 12211;  // IQ2/IR2: idum2 advances by jump-ahead
constexpr int NDIV = 1 + IMM1 / NTAB;
constexpr double AM = 1.0 / IM1;
constexpr double RNMX = 1.0 - 1.2e-7;
constexpr double kSqrt2Pi = 2.5066282746;  // mcmc_wrapper2.h:10
constexpr int kBlk = 64;                   // slots per workgroup of the gather kernel
#ifndef HB_DS_KPW
#define HB_DS_KPW 4
#endif
constexpr int kPW = HB_DS_KPW;             // propose waves (one slot each) per workgroup
#ifndef HB_DS_SEG  // experiment knob: owned slots per swap segment
#define HB_DS_SEG 128
#endif
constexpr int kSegSlots = HB_DS_SEG;       // owned slots per swap segment (one ds_swap_seg workgroup)
constexpr int kSegThreads = 256;
constexpr int kMaxLevels = 64;             // swap dependency levels a schedule buffer holds (W = 65 536: ~13)

// run constants (kernel argument)
struct Params {
  int W, NPAST;
  int log_on;
  int pad;
  double log_lc_period, LC_PERIOD;
  double lim_lo[kNp], lim_hi[kNp];  // limits[i]
  double fl_lo[kNp], fl_hi[kNp];    // limited[i] (1 reflecting, 2 periodic; doubles as in bounds)
  double sigma_p[kNp];
  int gpflag[kNp];
};

// Counters, Event, AccArgs: hb_accept.hpp

// one tempering attempt of the level schedule: pair (b, b+1) and ln(beta) of
// its acceptance draw (beta itself is kept in a global-only array beside it)
// schedule buffer of an iteration with nlv levels over G segments:
// int soff[G nlv + 1] | (8-B aligned) SwapEnt ent[nent] | double beta[nent];
// segment g's attempts of level l (0-based) are ent[soff[g nlv + l] ..
// soff[g nlv + l + 1]) -- an attempt near a segment border is listed for
// every segment whose cone holds its pair
__host__ __device__ inline size_t sched_ent_off(size_t G, size_t nlv) {
  return (sizeof(int) * (G * nlv + 1) + 7) & ~(size_t)7;
}
__host__ __device__ inline size_t sched_beta_off(size_t G, size_t nlv, size_t nent) {
  return sched_ent_off(G, nlv) + sizeof(SwapEnt) * nent;
}
__host__ __device__ inline size_t sched_bytes(size_t G, size_t nlv, size_t nent) {
  return sched_beta_off(G, nlv, nent) + sizeof(double) * nent;
}


// device state (pointers into one allocation set)
struct Dev {
  const Params* P; // run constants (device copy)
  int lo, nl;      // owned slots [lo, lo + nl); arrays "by slot" below are local (j - lo)
  double* hs;      // [W] tempering factor of the pair (b, b+1): (T_b - T_b+1) / (T_b T_b+1)
  double* x;       // [W][21] by chain
  double* logL;    // [W] by chain
  double* logP;    // [W] by chain
  int* logP_ok;    // [W] by chain
  int* idx;        // [W] slot -> chain (the current iteration's)
  int* idx_out;    // [W] the other buffer: ds_swap_seg writes the next iteration's index[] there
  int* order;      // [nl] propose wave -> (global) slot, hottest rungs first (dispatch order)
  int* ecnt;       // [kOrdBins] proposals per e bin (AccArgs::ecnt; null: eval waves in slot order)
  int* ecnt_next;  // the other buffer (the next iteration's; cleared by this iteration's Hastings launch)
  int par;         // the iteration's parity (Counters::de_trial_pend slot), counted by the host
  long long* nsw;  // [nl] accepted swaps with b = slot counted by deferred replays, folded into
                   // Counters::nswap by the next ds_swap_seg (no same-address atomics per wave)
  int* elist;      // [kOrdBins][nl] local slots by e bin
  double* wc;      // [nl] WalkerConst records (the context's workspace; set per launch)
  hbk::MagArgs ma; // Gaia term data of the context
  const double* tab_pc;  // period of the context's phase table (NaN: none)
  double* temp;    // [W]
  int* idum;       // [nl] ran2 state by slot
  int* idum2;
  int* iy;
  int* iset;
  double* gset;
  long long* cts;
  int* iv;         // [nl][32] (shuffle table row per slot)
  double* y;       // [nl][21] proposals by slot
  double* logPy;   // [nl]
  double* alpha2;  // [nl]
  double* logLy;   // [nl]
  int* jump;       // [nl]
  int* jtype;      // [nl]
  double* hist;    // [nl][NPAST][21] by slot
  int* DEacc_arr;  // [nl]
  int* DEtrial_arr;
  Counters* ctr;
  Event* ev;
};

// ---------------------------------------------------------------------------
// ran2_parallel / gasdev2_parallel (:894-974) for one slot per wave
// ---------------------------------------------------------------------------
// The stream of a slot is a fixed sequence of integers; which draws become
// uniforms, polar attempts or DE indices only decides how many are consumed.
// ran2 is two L'Ecuyer LCGs plus a Bays-Durham shuffle.  The LCG terms of
// draw base + k come lane-parallel by jump-ahead (lane k multiplies the base
// state by IA^(k+1) mod IM, a constant table); Schrage's product (:919-925)
// is the exact residue, and so is the modular product here.  Only the shuffle
// (iy -> table slot -> iy) is serial: it runs in scalar registers with the
// 32-entry table in one VGPR (lane t = iv[t], read by v_readlane, written by
// a lane select), on demand, into a 64-draw window (lane k = draw base + k).
// The transforms then run lane-parallel: up to 32 polar attempts at once,
// log / sqrt / division only on the accepted ones.  The state handed back is
// the state after exactly the consumed draws: the table at the window base is
// advanced by replaying the consumed draws' writes (slot iy_(k-1) / NDIV,
// value idum_k).
__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// a wave-uniform int the compiler cannot prove uniform: pin it to an SGPR so
// loops over it stay scalar (s_cbranch) instead of exec-mask loops
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// lane l of old := v (uniform v, l); a compare + select, so the compiler owns the SGPR hazards
__device__ __forceinline__ int wl(int v, int l, int old) { return (int)(threadIdx.x & 63) == l ? v : old; }
__device__ __forceinline__ double rld(double v, int l) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)rl((int)(uint32_t)u, l), hi = (uint32_t)rl((int)(uint32_t)(u >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int shfli(int v, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ double uni_of(int iy) {  // ran2's return value (:940-941)
  const double temp = AM * (double)iy;
  return temp > RNMX ? RNMX : temp;
}
__device__ __forceinline__ int ndiv(int iy) { return (int)((unsigned)iy / (unsigned)NDIV); }  // iy >= 1

// IA^(k+1) mod IM, k < 64, for both generators
struct LcgPow {
  int a1[64], a2[64];
};
constexpr LcgPow make_lcg_pow() {
  LcgPow t{};
  long long p1 = 1, p2 = 1;
  for (int k = 0; k < 64; ++k) {
    p1 = p1 * IA1 % IM1;
    p2 = p2 * IA2 % IM2;
    t.a1[k] = (int)p1;
    t.a2[k] = (int)p2;
  }
  return t;
}
__constant__ LcgPow kLcgPow = make_lcg_pow();

// a * z mod (2^31 - c) for 0 <= a, z < 2^31 - c: two folds of the high bits
// (2^31 = c mod m), one conditional subtraction
template <unsigned C>
__device__ __forceinline__ int mulmod31(int a, int z) {
  uint64_t x = (uint64_t)(uint32_t)a * (uint32_t)z;
  x = (x >> 31) * C + (x & 0x7fffffffu);
  x = (x >> 31) * C + (x & 0x7fffffffu);
  uint32_t r = (uint32_t)x;
  const uint32_t m = 0x80000000u - C;
  if (r >= m) r -= m;
  return (int)r;
}
static_assert(IM1 == 2147483648LL - 85 && IM2 == 2147483648LL - 249, "moduli are 2^31 - c");

struct WaveStream {
  // window base: the state after the last consumed draw (wave-uniform; table in a VGPR)
  int b_idum, b_idum2, b_iy, b_tab;
  // generator head: the shuffle state after draw base + gend - 1
  int g_iy, g_tab;
  // lane k: LCG states (idum, idum2) of draw base + k (all lanes) and its iy (k < gend)
  int w_idum, w_idum2, w_iy;
  int gend;            // generated draws in the window
  int cur;             // next unconsumed lane (uniform)
  long long consumed;  // draws consumed this kernel (cts increment)

  __device__ void jump() {  // LCG lanes from the base state
    const int k = threadIdx.x & 63;
    w_idum = mulmod31<85>(kLcgPow.a1[k], b_idum);
    w_idum2 = mulmod31<249>(kLcgPow.a2[k], b_idum2);
  }
  __device__ void gen_to(int n) {  // the serial shuffle for lanes gend .. n-1
    n = uni(n);
    int iy = uni(g_iy);
    for (int k = uni(gend); k < n; ++k) {
      const int j = uni(ndiv(iy));
      iy = uni(rl(g_tab, j) - rl(w_idum2, k));
      g_tab = wl(rl(w_idum, k), j, g_tab);
      if (iy < 1) iy += IMM1;
      w_iy = wl(iy, k, w_iy);
    }
    g_iy = iy;
    gend = uni(max(n, gend));
  }
  // start from (idum, idum2, iy, table); the table initialisation of
  // :905-916 runs here when idum <= 0 (a propose always consumes draws)
  __device__ void init(int idum, int idum2, int iy, int tab) {
    if (idum <= 0) {
      idum = (-idum < 1) ? 1 : -idum;
      idum2 = idum;
      for (int j = NTAB + 7; j >= 0; --j) {
        const int q = idum / IQ1;
        idum = IA1 * (idum - q * IQ1) - q * IR1;
        if (idum < 0) idum += IM1;
        if (j < NTAB) tab = wl(idum, j, tab);
      }
      iy = rl(tab, 0);
    }
    b_idum = idum;
    b_idum2 = idum2;
    g_iy = b_iy = iy;
    g_tab = b_tab = tab;
    w_iy = 0;
    gend = cur = 0;
    consumed = 0;
    jump();
  }
  // retire lanes 0..cur-1: the base state advances past them, the window slides down
  __device__ void slide() {
    const int s = uni(cur);
    if (s == 0) return;
    int prev = uni(b_iy);
    for (int k = 0; k < s; ++k) {
      b_tab = wl(rl(w_idum, k), uni(ndiv(prev)), b_tab);
      prev = rl(w_iy, k);
    }
    b_iy = prev;
    b_idum = rl(w_idum, s - 1);
    b_idum2 = rl(w_idum2, s - 1);
    w_iy = shfli(w_iy, min((int)(threadIdx.x & 63) + s, 63));
    gend = uni(gend - s);
    consumed += s;
    cur = 0;
    jump();
  }
  __device__ double uniform() {  // one ran2() call
    cur = uni(cur);
    if (cur == 64) slide();
    if (cur >= uni(gend)) gen_to(min(64, cur + 8));
    return uni_of(rl(w_iy, cur++));
  }
  __device__ int idum_now() const { return cur == 0 ? b_idum : rl(w_idum, cur - 1); }
};

// gaussian() (:1175-1178) and get_logP (:703-765)
__device__ double gauss_pdf(double x, double mean, double sigma, const hbglibc::Tabs& T) {
  return (1 / sigma / kSqrt2Pi) * hbglibc::exp(-hbglibc::pow((x - mean) / sigma, 2., T) / 2., T);
}

// one term of get_logP (:703-765): log(gaussian(x_i, mean_i, sigma_i))
__device__ double prior_term(int i, double xi, const hbglibc::Tabs& T) {
  double mean, sig;
  if (i == 7 || i == 8) { mean = 0.; sig = 1.; }
  else if (i == 9 || i == 11) { mean = 0.16; sig = 0.04; }
  else if (i == 10 || i == 12) { mean = 0.34; sig = 0.04; }
  else if (i == 13 || i == 14) { mean = 1.; sig = 0.2; }
  else if (i == 15 || i == 16) { mean = 0.; sig = 0.1; }
  else if (i == 17 || i == 18) { mean = 0.; sig = 1.; }
  else { mean = 0.; sig = 1.e15; }
  return hbglibc::log(gauss_pdf(xi, mean, sig, T), T);
}

// kNp successive gasdev2_parallel() values (:947-974); lane n < kNp gets
// value n.  iset/gset are the slot's Gaussian carry (wave-uniform).  Each
// round tests up to 32 polar attempts (draws 2m, 2m+1 of the window) at once.
__device__ double gauss_batch(WaveStream& S, int& iset, double& gset, const hbglibc::Tabs& T, double* gs) {
  const int lane = threadIdx.x & 63;
  int pos = 0;
  if (S.idum_now() < 0) iset = 0;  // :951
  if (iset) {
    if (lane == 0) gs[0] = gset;
    pos = 1;
    iset = 0;
  }
  while (pos < kNp) {
    S.slide();
    const int need = uni((kNp - pos + 1) / 2);          // pairs still to generate
    const int att = uni(min(32, need + need / 2 + 2));  // attempts tested this round (acceptance pi/4)
    S.gen_to(2 * att);
    const int m = lane & 31;
    const double v1 = 2.0 * uni_of(shfli(S.w_iy, 2 * m)) - 1.0;
    const double v2 = 2.0 * uni_of(shfli(S.w_iy, 2 * m + 1)) - 1.0;
    const double rsq = v1 * v1 + v2 * v2;
    const bool ok = lane < att && !(rsq >= 1.0 || rsq == 0.0);
    const uint64_t mask = __ballot(ok);
    const int avail = __popcll(mask);
    const int take = uni(min(need, avail));
    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    double g1 = 0.0;
    if (ok && rank < take) {
      const double fac = sqrt(-2.0 * hbglibc::log(rsq, T) / rsq);
      g1 = v1 * fac;
      const int o = pos + 2 * rank;
      gs[o] = v2 * fac;
      if (o + 1 < kNp) gs[o + 1] = g1;
    }
    if (take > 0) {
      // lane of the take-th accepted attempt: its v1 * fac is the new gset
      uint64_t mm = mask;
      for (int r = 1; r < take; ++r) mm &= mm - 1;
      const int last = uni(__builtin_ctzll(mm));
      gset = rld(g1, last);
      S.cur = (take == need) ? 2 * (last + 1) : 2 * att;
      const int got = 2 * take;
      if (take == need && pos + got > kNp) iset = 1;  // the last pair's v1 * fac is carried
      pos += got;
    } else {
      S.cur = 2 * att;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return lane < kNp ? gs[lane] : 0.0;
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// proposals (:386-485), one slot per wave, kPW waves per workgroup sharing the
// LDS copy of the exp/log/pow tables.  Lane n < 21 holds coordinate n of x
// and y; walls and prior terms run one coordinate per lane.  Wave w of block
// b takes slot order[kPW b + w], order = slots by descending temperature: the
// hot rungs' long wall runs are dispatched first, and a workgroup's waves
// (spread over its CU's SIMDs) share each SIMD with colder slots of the CU's
// later workgroups (measured 37.5 -> 35.2 us against order[b + w grid]).
// Epilogue: the workgroup's four waves become one prep group (hb_prep.hpp)
// and write the likelihood's per-walker records of their slots, and each
// slot is filed under its e bin for the eval launch's order -- the likelihood
// launch follows directly, with no prep launch in between.
// The iteration's swap schedule (n8 words) is copied from the pinned ring
// entry into its device ring entry on the way (the coldest slots' waves, which
// finish first, issue the reads; system-scope loads bypass the GPU caches),
// so ds_swap depends on nothing outside this stream: a separate copy stream
// cost an inter-queue event wait of ~10 us per iteration before ds_swap.
// PREP = false (more slots than one resident round of 4 waves per SIMD): the
// epilogue's ~100 VGPRs would halve the kernel's occupancy (64 VGPRs, 7 waves
// per SIMD without it), so the records come from a separate hb_prep_kernel
// launch instead.
static_assert(kPW == hbk::kPrepRoles, "the propose workgroup is one prep group");
#ifndef HB_DS_PROPOSE_WPE
#define HB_DS_PROPOSE_WPE 0  // > 0: minimum waves per SIMD for ds_propose (experiment builds)
#endif
#if HB_DS_PROPOSE_WPE > 0
#define HB_DS_PROPOSE_ATTR __attribute__((amdgpu_waves_per_eu(HB_DS_PROPOSE_WPE)))
#else
#define HB_DS_PROPOSE_ATTR
#endif
// LDS of a propose workgroup (ds_propose)
struct ProposeShared {
  uint64_t tab[hbglibc::kTabWords];  // exp / log / pow tables (divergent lookups)
  double gs[kPW][32];
  hbk::PrepShared<kPW> PL;
  int jl[kPW];
};
#ifdef HB_DS_CLOCKS
// experiment builds only: per slot of the last propose: the phase stamps DS_T(0..7) (s_memtime), s_memrealtime at
// entry and after the stores, its temperature, proposal type (hb_debug_dp_clocks)
constexpr int kDpClkWords = 16;
__device__ unsigned long long dp_clk[kDpClkWords * 65536];
#endif
// the per-iteration bookkeeping after the swaps (:551-572, :590, :622-629)
// by thread 0 of one workgroup; c0 = the chain now in slot 0 (-1: not this
// rank's slot).  nswap is added by every segment (atomics).
__device__ __forceinline__ void swap_tail(const Dev& D, long long iter, int par, int c0) {
  Counters* C = D.ctr;
  C->DEtrial_tot += C->de_trial_pend[par];  // the iteration's proposals' DE trials (Counters)
  C->de_trial_pend[par] = 0;
  C->acc += C->acc_it;  // hb_sampler_accept's sums over the slots
  C->cold_acc += C->acc_it;
  C->DEacc += C->DEacc_tot;
  C->DEtrial += C->DEtrial_tot;
  C->acc_it = 0;
  C->snap[0] = C->acc;
  C->snap[1] = C->DEacc;
  C->snap[2] = C->DEtrial;
  C->snap[3] = C->atrial;
  if (c0 >= 0 && D.logL[c0] > C->logLmap) {  // :565-572
    for (int i = 0; i < kNp; ++i) C->xmap[i] = D.x[(size_t)c0 * kNp + i];
    C->logLmap = D.logL[c0];
  }
  C->atrial++;  // :590 and the 100-step reset of :622-629
  if (iter % 100 == 0) {
    C->acc = C->atrial = 0;
    C->DEacc_tot = C->DEtrial_tot = 0;
  }
}

// The previous iteration's tempering swaps, deferred from their own launch
// into this ds_propose (one-process samplers, hb_dsampler::pend): the wave of
// slot j replays the cone of the one-slot segment [j, j + 1), i.e. the
// attempts whose pair lies in [j - nlv, j + nlv + 1), taken from the attempt
// lists of the ds_swap_seg segment holding j (whose cone contains it).  The
// segment argument of ds_swap_seg holds for a one-slot segment: after the nlv
// levels slot j's chain is exact, and so is every attempt with b = j, which
// the wave counts (nswap).  So slot j's chain needs no other wave and no
// launch boundary: it is written to this iteration's index[] (idx_out) and
// the proposal reads its state.  The iteration's bookkeeping (swap_tail) is
// run by slot 0's wave.
struct SwapPrev {
  const int* soff;        // the previous iteration's schedule (its device ring slot)
  const SwapEnt* ent;
  const double* betas;
  const double* Ls;       // [W] logL by slot after the previous Hastings test (null: D.logL by chain)
  int* idx_out;           // [W] this iteration's index[]
  long long iter;         // the previous iteration
  int nlv, G;
  int cone, maxent;       // per-wave LDS sizing: cone slots (2 nlv + 1), attempts of one segment
};
__host__ __device__ inline size_t swap_prev_wave_bytes(int cone, int maxent) {
  return (((size_t)cone * (2 * sizeof(double) + sizeof(int)) + 15) & ~(size_t)15) + sizeof(SwapEnt) * (size_t)maxent;
}
// The replay's global loads, issued before ds_propose's table-staging barrier
// so that their two dependent rounds (the segment's level offsets, then its
// attempts) overlap the tables, the slot state and the barrier instead of
// starting after them: the cone's first 64 slots (chain, hs, logL) and the
// offsets (replay_load_cone, right after the slot is known), then the first
// kRpEnts x 64 attempts (replay_load_ents, just before the barrier).
constexpr int kRpEnts = 4;
struct ReplayLoads {
  int g, so, c;   // segment; lane <= nlv: level lane's first attempt; lane < Wc: the cone slot's chain
  double h, L;    // lane < Wc: the slot's inverse-temperature difference and logL
  int eb, eend;   // the segment's attempts [eb, eend)
  int eb_[kRpEnts];     // attempts eb + lane + 64 r: b and ln(beta) (scalars, not a SwapEnt
  double el_[kRpEnts];  // array: that one went to scratch)
};
__device__ __forceinline__ void replay_load_cone(const Dev& D, const SwapPrev& SP, int W, int j, int lane,
                                                 ReplayLoads& R) {
  const int nlv = SP.nlv;
  R.g = seg_of(j - D.lo, D.nl, SP.G);
  const int clo = max(0, j - nlv), Wc = min(W, j + nlv + 1) - clo;
  R.so = lane <= nlv ? SP.soff[R.g * nlv + lane] : 0;
  R.c = 0;
  R.h = R.L = 0.0;
  if (lane < Wc) {
    R.c = D.idx[clo + lane];
    R.h = D.hs[clo + lane];
    R.L = SP.Ls != nullptr ? SP.Ls[clo + lane] : D.logL[R.c];
  }
}
__device__ __forceinline__ void replay_load_ents(const SwapPrev& SP, int lane, ReplayLoads& R) {
  const int nlv = SP.nlv;
  R.eb = __builtin_amdgcn_readfirstlane(R.so);
  R.eend = nlv < 64 ? __builtin_amdgcn_readlane(R.so, nlv) : SP.soff[R.g * nlv + nlv];
  const int ne = R.eend - R.eb;
#pragma unroll
  for (int r = 0; r < kRpEnts; ++r) {
    const int q = lane + 64 * r;
    int b = 0;
    double l = 0.0;
    if (q < ne) {
      const SwapEnt x = SP.ent[R.eb + q];
      b = x.b;
      l = x.lnb;
    }
    R.eb_[r] = b;
    R.el_[r] = l;
  }
}
// returns the chain in slot j after the previous iteration's swaps; nacc: the
// accepted attempts with b = j (wave-uniform); R: the loads issued ahead
// (replay_load_cone / replay_load_ents)
__device__ __forceinline__ int replay_prev_swaps(const Dev& D, const SwapPrev& SP, int W, int j, int lane,
                                                 const hbglibc::Tabs& T, unsigned char* scr, int& nacc,
                                                 const ReplayLoads& R, unsigned long long* rp = nullptr) {
  if (rp) rp[0] = __builtin_amdgcn_s_memtime();
  const int nlv = SP.nlv;
  const int clo = max(0, j - nlv), chi = min(W, j + nlv + 1), Wc = chi - clo;
  double* cL = reinterpret_cast<double*>(scr);
  double* cH = cL + SP.cone;
  int* cC = reinterpret_cast<int*>(cH + SP.cone);
  SwapEnt* sE = reinterpret_cast<SwapEnt*>(scr + (((size_t)SP.cone * (2 * sizeof(double) + sizeof(int)) + 15) &
                                                  ~(size_t)15));
  // the segment's level offsets (nlv + 1 <= 65 of them: lane l holds level l's
  // start, lane 64 the end read apart), its attempts and the cone's slots
  const int so = R.so;
  if (lane < Wc) {
    cC[lane] = R.c;
    cH[lane] = R.h;
    cL[lane] = R.L;
  }
  for (int i = lane + 64; i < Wc; i += 64) {  // cones wider than a wave (nlv >= 32)
    const int c = D.idx[clo + i];
    cC[i] = c;
    cH[i] = D.hs[clo + i];
    cL[i] = SP.Ls != nullptr ? SP.Ls[clo + i] : D.logL[c];
  }
  const int eb = R.eb, eend = R.eend;
  const int ne = eend - eb;
#pragma unroll
  for (int r = 0; r < kRpEnts; ++r)
    if (lane + 64 * r < ne) {
      sE[lane + 64 * r].b = R.eb_[r];
      sE[lane + 64 * r].lnb = R.el_[r];
    }
  for (int q = lane + 64 * kRpEnts; q < ne; q += 64) sE[q] = SP.ent[eb + q];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (rp) {
    rp[1] = __builtin_amdgcn_s_memtime();
    rp[3] = (unsigned long long)(unsigned)ne | ((unsigned long long)(unsigned)nlv << 32);
  }
  int acc_j = 0;
  for (int lv = 0; lv < nlv; ++lv) {  // ds_swap_seg's level loop on the cone's attempts
    const int e0 = __builtin_amdgcn_readlane(so, lv) - eb;
    const int e1 = (lv + 1 < 64 ? __builtin_amdgcn_readlane(so, lv + 1) : eend) - eb;
    for (int q = e0 + lane; q < e1; q += 64) {
      const int b = sE[q].b;
      if (b < clo || b + 1 >= chi) continue;  // its pair is not in this slot's cone
      const double lnb = sE[q].lnb;
      const int bl = b - clo, al = bl + 1;
      const double lb = cL[bl], la = cL[al];
      const double x = (lb - la) * cH[bl];
      bool acc;
      const double dl = 1e-12 * (1.0 + fabs(lnb));
      if (lnb > -HUGE_VAL && x >= lnb + dl) acc = true;
      else if (lnb > -HUGE_VAL && x <= lnb - dl) acc = false;
      else acc = hbglibc::exp(x, T) >= SP.betas[eb + q];
      if (acc) {
        const int ca = cC[al], cb = cC[bl];
        cL[al] = lb;
        cL[bl] = la;
        cC[al] = cb;
        cC[bl] = ca;
        if (b == j) ++acc_j;  // a pair may be attempted at several levels
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (rp) rp[2] = __builtin_amdgcn_s_memtime();
  for (int off = 32; off >= 1; off >>= 1) acc_j += __shfl_xor(acc_j, off, 64);
  nacc = __builtin_amdgcn_readfirstlane(acc_j);
  return __builtin_amdgcn_readfirstlane(cC[j - clo]);
}

// the body of ds_propose: every wave of the workgroup calls it (it holds the
// prep group's barriers); j_out: the wave's global slot, act_out: whether it
// has one (the grid's last workgroup may hold fewer than kPW).  SWAP: the
// previous iteration's swaps replayed first (SwapPrev; scr: the wave's LDS)
template <bool PREP, bool SWAP = false>
__device__ __forceinline__ void propose_group(const Dev& D, int W, int NPAST, long long iter,
                                              const unsigned long long* __restrict__ sch_src,
                                              unsigned long long* __restrict__ sch_dst, long long n8,
                                              ProposeShared& Ls, int& j_out, bool& act_out,
                                              const SwapPrev& SP = SwapPrev{}, unsigned char* scr = nullptr) {
  const long long sgt = (long long)(gridDim.x - 1 - blockIdx.x) * blockDim.x + threadIdx.x;
  const long long sgs = (long long)gridDim.x * blockDim.x;
  unsigned long long sv = 0;
  if (sgt < n8) sv = __hip_atomic_load(sch_src + sgt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  uint64_t* tab_s = Ls.tab;
  hbk::PrepShared<kPW>& PL = Ls.PL;
  int* jl_s = Ls.jl;
  const Params* P = D.P;
  const hbglibc::Tabs T{tab_s, tab_s + 256, tab_s + 512};
  {
    const hbglibc::Tabs C = hbglibc::const_tabs();
    for (int q = threadIdx.x; q < 256; q += 64 * kPW) {
      tab_s[q] = C.exp[q];
      tab_s[256 + q] = C.log[q];
      tab_s[512 + q] = C.pow[q];
      tab_s[768 + q] = C.pow[256 + q];
    }
  }
  // the slot's state loads overlap the table staging; the barrier follows them
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int k = (int)blockIdx.x * kPW + wv;
  const bool act = k < D.nl;
  const int j = act ? D.order[k] : D.lo;  // global slot
  const int jl = j - D.lo;                // local slot (arrays by slot)
  double* gs = Ls.gs[wv];
  ReplayLoads rl;
  if constexpr (SWAP)
    if (act) replay_load_cone(D, SP, W, j, lane, rl);
  j_out = j;
  act_out = act;
  const double pc_tab = PREP ? *D.tab_pc : 0.0;
#ifdef HB_DS_CLOCKS  // experiment builds only: per-slot phase stamps (dp_clk, scripts/ds_clocks.py)
  unsigned long long tclk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long rp_[4] = {0, 0, 0, 0};  // deferred-swap replay: start, staged, levels done, (ne | nlv << 32)
  const unsigned long long trt0 = __builtin_amdgcn_s_memrealtime();
#define DS_T(k) tclk[k] = __builtin_amdgcn_s_memtime()
#define DS_PRINT()                                                                      \
  if (jl < 65536) {                                                                     \
    unsigned long long* o_ = dp_clk + kDpClkWords * jl;                                 \
    for (int q_ = 0; q_ < 8; ++q_) o_[q_] = tclk[q_];                                   \
    o_[8] = trt0;                                                                       \
    o_[9] = __builtin_amdgcn_s_memrealtime();                                           \
    o_[10] = (unsigned long long)__double_as_longlong(temp);                            \
    o_[11] = (unsigned long long)(jt | (jmp << 8));                                     \
    o_[12] = rp_[0];                                                                    \
    o_[13] = rp_[1];                                                                    \
    o_[14] = rp_[2];                                                                    \
    o_[15] = rp_[3];                                                                    \
  }
#else
#define DS_T(k)
#define DS_PRINT()
#endif
  DS_T(0);
  // SWAP: the chain in slot j before the previous iteration's swaps, its
  // state loaded ahead and kept when no accepted swap moved it (the replay)
  int chain = D.idx[j];
  bool needx = !D.logP_ok[chain];
  double xn = lane < kNp ? D.x[(size_t)chain * kNp + lane] : 0.0;
  const double temp = D.temp[j];
  int iset = D.iset[jl];
  double gset = D.gset[jl];
  WaveStream S;
  S.init(D.idum[jl], D.idum2[jl], D.iy[jl], lane < NTAB ? D.iv[(size_t)jl * NTAB + lane] : 0);
  if constexpr (SWAP)
    if (act) replay_load_ents(SP, lane, rl);
  __syncthreads();  // tables staged
  if (sgt < n8) sch_dst[sgt] = sv;
  for (long long q = sgt + sgs; q < n8; q += sgs)
    sch_dst[q] = __hip_atomic_load(sch_src + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if constexpr (SWAP) {
    if (act) {  // the previous iteration's swaps for this slot, then its state
      int nacc = 0;
#ifdef HB_DS_CLOCKS
      unsigned long long* rpp = rp_;
#else
      unsigned long long* rpp = nullptr;
#endif
      const int c1 = replay_prev_swaps(D, SP, W, j, lane, T,
                                       scr + (size_t)wv * swap_prev_wave_bytes(SP.cone, SP.maxent), nacc, rl, rpp);
      if (lane == 0) {
        SP.idx_out[j] = c1;
        if (nacc) D.nsw[jl] += nacc;  // this slot's own counter: no contention
        if (SP.iter % 100 == 0) D.DEacc_arr[jl] = D.DEtrial_arr[jl] = 0;  // ds_swap_seg's 100-step reset
        if (j == 0) swap_tail(D, SP.iter, D.par ^ 1, c1);  // slot 0 (one-process samplers own every slot)
      }
      if (c1 != chain) {  // wave-uniform
        chain = c1;
        needx = !D.logP_ok[chain];
        xn = lane < kNp ? D.x[(size_t)chain * kNp + lane] : 0.0;
      }
    }
  }
  if (act) {  // wave-uniform; every wave reaches the prep group's barriers below
    DS_T(1);
    const double a = S.uniform();
    DS_T(2);
    const double jscale = hbglibc::pow(10., -6. + 6. * a, T);
    int jmp = 0, jt = 0;
    if ((S.uniform() < 0.5) && (iter > NPAST)) jmp = 1;
    double yn = xn;
    // gaussian_proposal_parallel (:1062-1088)
    auto gaussian_step = [&]() {
      const double sqtemp = sqrt(temp);
      const double g = gauss_batch(S, iset, gset, T, gs);
      if (lane < kNp) yn = xn + g * P->sigma_p[lane] * sqtemp * jscale;
    };
    if (jmp == 0) {
      gaussian_step();
      jt = 1;
    }
    if (jmp == 1) {
      if (chain == 0 && lane == 0) {
        D.DEtrial_arr[jl]++;
        atomicAdd((unsigned long long*)&D.ctr->de_trial_pend[D.par], 1ull);
      }
      // differential_evolution_proposal_parallel (:1091-1140) as compiled (see
      // hb_sampler.cpp de_step: a == 0, the uninitialised c == 0).  The 0.9
      // draw precedes the per-parameter Gaussians, as in the reference.
      int ia = (int)(S.uniform() * NPAST);
      ia = (int)S.uniform();
      int ib = ia;
      while (ib == ia) ib = (int)(S.uniform() * NPAST);
      // gaussian(c = 0, 0, 1e-4) - 0.5 (:1115): pow(0, 2) = 0 and exp(-0) = 1
      // exactly, so gauss_pdf's value is its constant factor, folded here
      const double g0 = (1 / 1.e-4 / kSqrt2Pi) * 1.0 - 0.5;
      const bool scaled = S.uniform() < 0.9;
      const double gamma = 2.388 / sqrt(2. * kNp);  // GAMMA, mcmc_wrapper2.h:13
      const double gd = scaled ? gauss_batch(S, iset, gset, T, gs) : 0.0;
      if (lane < kNp) {
        const double* hist = &D.hist[(size_t)jl * NPAST * kNp];
        double dx = hist[(size_t)ib * kNp + lane] - hist[(size_t)ia * kNp + lane];
        const double eps = dx * g0;
        if (scaled) dx *= gd * gamma;
        dx += eps;
        yn = xn + dx;
      }
      jt = 2;
      double dx_mag = 0;  // summed in coordinate order
      const double d = xn - yn;
      for (int i = 0; i < kNp; ++i) {
        const double di = rld(d, i);
        dx_mag += di * di;
      }
      if (dx_mag < 1e-6) {
        gaussian_step();
        jt = 1;
      }
    }
    DS_T(3);
    DS_T(4);
    // A proposal with e > 1 that the walls leave as it is (e has no upper
    // wall, set_limits :986-1121) gets a NaN logL whatever its other
    // coordinates (hb_device.hpp logl_without_light_curve: 1 - e^2 < 0, Roche
    // impossible with the periastron a (1 - e) < 0), so the Hastings test
    // rejects it.  Its other coordinates' walls and its prior terms feed only
    // that logL, the records and the test, and a rejected proposal is never
    // stored: they are skipped (logPy = NaN).  No draw depends on them.
    const double e_pre = rld(yn, 3);
    const bool e_kept = (e_pre >= P->lim_lo[3] || (P->fl_lo[3] != 1 && P->fl_lo[3] != 2)) &&
                        (e_pre <= P->lim_hi[3] || (P->fl_hi[3] != 1 && P->fl_hi[3] != 2));  // the walls leave e alone
    const bool lost = e_pre > 1.0 && e_kept;  // profiles/r05/r05p_ds_lost_acc_ab.txt
    // walls (:440-467), one coordinate per lane.  A slot whose proposal lands
    // many ranges outside (the hot rungs) folds for thousands of cycles, a
    // dependent chain that sets the launch's tail: its wave takes issue
    // priority over the throughput-bound waves beside it for the duration
#ifndef HB_DS_WALL_PRIO
#define HB_DS_WALL_PRIO 1
#endif
    const bool wfar = HB_DS_WALL_PRIO && __ballot(lane < kNp && (!lost || lane == 3) &&
                                                  fabs(yn - 0.5 * (P->lim_lo[lane] + P->lim_hi[lane])) >
                                                      8.0 * (P->lim_hi[lane] - P->lim_lo[lane])) != 0;
    if (wfar) __builtin_amdgcn_s_setprio(3);
    if (lane < kNp && (!lost || lane == 3))
      yn = hbwall::apply_wall(yn, P->lim_lo[lane], P->lim_hi[lane], P->fl_lo[lane], P->fl_hi[lane]);
    if (wfar) __builtin_amdgcn_s_setprio(0);
    // "order the masses" (:470-475) as written: y[1] = y[0]; period fixed; T0 folded
    const double y0 = rld(yn, 0), y1 = rld(yn, 1);
    if (lane == 1 && y1 > y0) yn = y0;
    if (lane == 2) yn = P->log_lc_period;
    if (lane == 6) yn = fmod(yn, P->LC_PERIOD);
    // the e-bin slot (the eval order, hbds::eval_slot_by_e): e is final here,
    // so the returning atomic's latency overlaps the prior terms
    int ebin = 0, eslot = 0;
    if (lane == 3 && D.ecnt != nullptr) {
      ebin = e_bin_desc(yn);
      eslot = atomicAdd(&D.ecnt[ebin * kEbinStride], 1);
    }
    DS_T(5);
    // prior terms (:444, :477), summed per slot in the reference's order
    const bool prior = lane < kNp && P->gpflag[lane] == 1;
    const double ty = (prior && !lost) ? prior_term(lane, yn, T) : 0.0;
    const double tx = (needx && prior) ? prior_term(lane, xn, T) : 0.0;
    double lpy = 0., lpx = 0.;
    const uint64_t pmask = __ballot(prior);  // the flags as one mask: no scalar load per term
    for (int i = 0; i < kNp; ++i) {
      if (!((pmask >> i) & 1u)) continue;
      lpy += rld(ty, i);
      if (needx) lpx += rld(tx, i);
    }
    if (lost) lpy = __builtin_nan("");
    DS_T(6);
    // the alpha draw and the retirement of the consumed draws only feed the
    // stored state, so they follow the walls (off the hot slots' critical path)
    const double alpha2 = S.uniform();  // drawn after the likelihood calls in the reference; same stream order
    S.slide();
    if (lane < kNp) {
      D.y[(size_t)jl * kNp + lane] = yn;
      if (PREP) PL.sp[wv * hbk::kNpars + lane] = yn;
    }
    if (lane == 3 && D.ecnt != nullptr) D.elist[(size_t)ebin * D.nl + eslot] = jl;
    if (lane < NTAB) D.iv[(size_t)jl * NTAB + lane] = S.b_tab;
    if (lane == 0) {
      jl_s[wv] = jl;
      D.logPy[jl] = lpy;
      if (needx) {
        D.logP[chain] = lpx;
        D.logP_ok[chain] = 1;
      }
      D.jump[jl] = jmp;
      D.jtype[jl] = jt;
      D.alpha2[jl] = alpha2;
      D.idum[jl] = S.b_idum;
      D.idum2[jl] = S.b_idum2;
      D.iy[jl] = S.b_iy;
      D.iset[jl] = iset;
      D.gset[jl] = gset;
      D.cts[jl] += S.consumed;
      DS_T(7);
      DS_PRINT();
    }
  }
  if (!PREP) return;
  // the likelihood's per-walker records of the group's slots: every wave
  // reads the others' proposals from PL.sp
  const int nb = min(kPW, D.nl - (int)blockIdx.x * kPW);
  __syncthreads();
  hbk::prep_records<kPW>(PL, nb, D.ma, nullptr, nullptr, 0, [&](int) { return pc_tab; }, [] {});
  for (int q = threadIdx.x; q < nb * hbk::kWcDoubles; q += 64 * kPW) {
    const int w = q / hbk::kWcDoubles, f = q - w * hbk::kWcDoubles;
    D.wc[(size_t)jl_s[w] * hbk::kWcDoubles + f] = PL.so[w * hbk::kSoStride + f];
  }
}
template <bool PREP, bool SWAP>
__global__ __launch_bounds__(64 * kPW) HB_DS_PROPOSE_ATTR void ds_propose(Dev D, int W, int NPAST, long long iter,
                                                       const unsigned long long* __restrict__ sch_src,
                                                       unsigned long long* __restrict__ sch_dst, long long n8,
                                                       SwapPrev SP) {
  __shared__ ProposeShared S;
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];  // SWAP: kPW waves' cone scratch
  int j;
  bool act;
  propose_group<PREP, SWAP>(D, W, NPAST, iter, sch_src, sch_dst, n8, S, j, act, SP, dyn);
}

// Hastings test and history (:492-546); 64 slots per block (one lane each),
// the state and history rows copied by the whole block
constexpr int kAccThreads = 256;
__global__ __launch_bounds__(kAccThreads) void ds_accept(Dev D, int W, int NPAST, long long iter) {
  __shared__ int chain_s[64], acc_s[64];
  const int tid = threadIdx.x, lane = tid;
  if (blockIdx.x == 0 && D.ecnt_next != nullptr && tid < kOrdBins) D.ecnt_next[tid * kEbinStride] = 0;
  const int j0 = blockIdx.x * 64;  // local slots j0 .. j0 + nw - 1
  const int nw = min(64, D.nl - j0);
  const int k = (int)(iter - (iter / NPAST) * NPAST);
  if (lane < nw) {
    const int jl = j0 + lane, j = jl + D.lo;
    const int chain = D.idx[j];
    const double ly = D.logLy[jl], lx = D.logL[chain];
    const double* xc = &D.x[(size_t)chain * kNp];
    const double* yj = &D.y[(size_t)jl * kNp];
    const double H = hbglibc::exp((ly - lx) / D.temp[j] + (D.logPy[jl] - D.logP[chain]));
    const bool acc = D.alpha2[jl] <= H;
    chain_s[lane] = chain;
    acc_s[lane] = acc;
    if (acc) {
      if ((lx / ly <= 0.5) && (iter > 10000) && (j <= 5) && D.P->log_on) {
        const int e = atomicAdd(&D.ctr->nev, 1);
        if (e < kEvCap) {
          Event& ev = D.ev[e];
          ev.iter = iter;
          ev.chain = chain;
          ev.jtype = D.jtype[jl];
          ev.slot = j;
          ev.H = H;
          ev.alpha = D.alpha2[jl];
          ev.tmp = D.temp[j];
          ev.lx = lx;
          ev.ly = ly;
          ev.px = D.logP[chain];
          ev.py = D.logPy[jl];
          for (int i = 0; i < kNp; ++i) {
            ev.xo[i] = xc[i];
            ev.xn[i] = yj[i];
          }
        }
      }
      if (chain == 0) atomicAdd((unsigned long long*)&D.ctr->acc_it, 1ull);
      D.logL[chain] = ly;
      D.logP[chain] = D.logPy[jl];
      if ((D.jump[jl] == 1) && (chain == 0)) {
        D.DEacc_arr[jl]++;
        atomicAdd((unsigned long long*)&D.ctr->DEacc_tot, 1ull);
      }
    }
  }
  __syncthreads();
  // x[chain] = y (accepted), history row k = x[chain] (:533-546): every
  // element's load is issued before any store, so the block waits for one
  // memory round trip instead of one per element
  constexpr int kPer = (kNp * 64 + kAccThreads - 1) / kAccThreads;
  double v[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const int q = tid + r * kAccThreads;
    v[r] = 0.0;
    if (q < kNp * nw) {
      const int w = q / kNp, n = q % kNp;
      v[r] = acc_s[w] ? D.y[(size_t)(j0 + w) * kNp + n] : D.x[(size_t)chain_s[w] * kNp + n];
    }
  }
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const int q = tid + r * kAccThreads;
    if (q < kNp * nw) {
      const int w = q / kNp, n = q % kNp;
      if (acc_s[w]) D.x[(size_t)chain_s[w] * kNp + n] = v[r];
      D.hist[((size_t)(j0 + w) * NPAST + k) * kNp + n] = v[r];
    }
  }
}

// Sharded runs: what a rank contributes to the iteration's all-gather
// (doubles): logL of its slots (padded to m = the largest shard), then K = 2
// nlv records of kRec doubles {chain, logP, logP_ok, x[21]} -- the chains in
// the nlv slots at each edge of the shard (record k < nlv: local slot k;
// k >= nlv: local slot nl - 2 nlv + k), chain -1 where that slot does not
// exist (shards smaller than nlv).
constexpr int kRec = 3 + kNp;
constexpr int kPackThreads = 256;
__global__ __launch_bounds__(kPackThreads) void ds_pack(Dev D, double* __restrict__ send, int m, int nlv) {
  const int q = (int)blockIdx.x * kPackThreads + (int)threadIdx.x;
  if (q < m) {
    send[q] = q < D.nl ? D.logL[D.idx[D.lo + q]] : 0.0;
    return;
  }
  const int r = q - m;
  if (r >= 2 * nlv * kRec) return;
  const int k = r / kRec, f = r - k * kRec;
  const int jl = k < nlv ? k : D.nl - 2 * nlv + k;
  double v = f == 0 ? -1.0 : 0.0;
  if (jl >= 0 && jl < D.nl) {
    const int c = D.idx[D.lo + jl];
    v = f == 0 ? (double)c : f == 1 ? D.logP[c] : f == 2 ? (double)D.logP_ok[c] : D.x[(size_t)c * kNp + (f - 3)];
  }
  send[m + r] = v;
}

// what ds_swap_seg imports in a sharded run
struct Gathered {
  const double* G;  // [R][S]: each rank's ds_pack output
  long long S;      // doubles per rank
  int R, me, m;
  int pad;
};

// Tempering swaps (ptmcmc :768-817) and the iteration's bookkeeping, one
// workgroup per segment [sl, sh) of the owned slots.  A level moves a slot's
// content by one, so after the nlv levels the chains of [sl, sh) come from the
// cone [sl - nlv, sh + nlv), and the attempts left out of the cone can disturb
// only slots within nlv - 1 of its edges, never [sl, sh): the workgroup
// replays in LDS just the cone's attempts (listed per segment and level by the
// producer thread) on the cone's (logL, chain) pairs and writes the owned
// slots' chains into the other index[] buffer, so the neighbouring segments
// still read the iteration's index[] for their cones.  An attempt with b in
// [sl, sh) sees exact inputs at every level and counts there (nswap).  No
// workgroup replays more than kSegSlots + 2 nlv slots, so the swap step is a
// wide launch instead of one workgroup walking all W attempts.
// XCHG (sharded runs and the one-rank exchange path): logL by slot comes from
// the all-gather (the owner rank's block) and the chain ids of other ranks'
// slots from their edge records, which also carry the state and logL of a
// chain that moves into an owned slot.
template <bool XCHG>
__global__ __launch_bounds__(kSegThreads) void ds_swap_seg(Dev D, int W, const int* __restrict__ soff,
                                                            const SwapEnt* __restrict__ ent,
                                                            const double* __restrict__ betas, int nlv, int G,
                                                            long long iter, Gathered X, const double* __restrict__ Ls) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ unsigned long long nacc_s;
  __shared__ uint64_t exp_s[256];  // exp table for the divergent lookups of the band case
  const int tid = threadIdx.x, g = blockIdx.x;
  const int lo = D.lo, hi = D.lo + D.nl;
  const int sl = seg_lo(lo, D.nl, g, G), sh = seg_lo(lo, D.nl, g + 1, G);
  const int clo = max(0, sl - nlv), chi = min(W, sh + nlv), Wc = chi - clo;
  // LDS: the segment's attempts (all levels), then the cone's logL, pair
  // factors and chain ids -- staged with every load in flight, so a level
  // costs LDS round trips only
  const int eb = soff[g * nlv], ne = soff[g * nlv + nlv] - eb;
  SwapEnt* sE = reinterpret_cast<SwapEnt*>(smem);
  double* cL = reinterpret_cast<double*>(smem + sizeof(SwapEnt) * (size_t)ne);
  double* cH = cL + Wc;
  int* cC = reinterpret_cast<int*>(cH + Wc);
  for (int q = tid; q < 256; q += kSegThreads) exp_s[q] = hbglibc::kExpTab[q];
  for (int q = tid; q < ne; q += kSegThreads) sE[q] = ent[eb + q];
  for (int i = tid; i < Wc; i += kSegThreads) cH[i] = D.hs[clo + i];
  const hbglibc::Tabs T{exp_s, hbglibc::kLogTab, hbglibc::kPowTab};
  if (!XCHG) {
    for (int i = tid; i < Wc; i += kSegThreads) {
      const int c = D.idx[clo + i];
      cC[i] = c;
      cL[i] = Ls != nullptr ? Ls[clo + i] : D.logL[c];  // Ls: by slot, written by the fused Hastings test
    }
  } else {
    auto rlo = [&](int r) { return (int)((long long)W * r / X.R); };
    for (int i = tid; i < Wc; i += kSegThreads) {
      const int s = clo + i;
      int r = (int)(((long long)s * X.R) / W);
      while (r + 1 < X.R && rlo(r + 1) <= s) ++r;
      while (r > 0 && rlo(r) > s) --r;
      cL[i] = X.G[(size_t)r * X.S + (s - rlo(r))];
      if (s >= lo && s < hi) cC[i] = D.idx[s];
    }
    // the other ranks' edge records inside the cone: chain id by slot, and the
    // chain's record and logL for the case it moves into an owned slot (two
    // segments whose cones share a record write the same values)
    const int nrec = (int)((X.S - X.m) / kRec), ke = nrec / 2;
    for (int r = 0; r < X.R; ++r) {
      if (r == X.me) continue;
      const int lo_r = rlo(r), nl_r = rlo(r + 1) - lo_r;
      if (lo_r >= chi || lo_r + nl_r <= clo) continue;
      const double* gr = X.G + (size_t)r * X.S + X.m;
      for (int q = tid; q < nrec * kRec; q += kSegThreads) {
        const int kk = q / kRec, f = q - kk * kRec;
        const int c = (int)gr[(size_t)kk * kRec];
        if (c < 0) continue;
        const int slot = lo_r + (kk < ke ? kk : nl_r - 2 * ke + kk);
        if (slot < clo || slot >= chi) continue;
        const double v = gr[q];
        if (f == 0) {
          cC[slot - clo] = c;
          D.logL[c] = X.G[(size_t)r * X.S + (slot - lo_r)];
        } else if (f == 1) {
          D.logP[c] = v;
        } else if (f == 2) {
          D.logP_ok[c] = (int)v;
        } else {
          D.x[(size_t)c * kNp + (f - 3)] = v;
        }
      }
    }
  }
  if (tid == 0) nacc_s = 0ull;
  __syncthreads();
  // the levels.  One attempt (:782-812): exp(x) >= beta decided by x against
  // ln(beta) outside a band of 1e-12 (1 + |ln beta|), far wider than the ulp
  // errors of the host log and of exp; inside the band (or beta = 0, NaN x)
  // the glibc-exact exp is compared with beta itself
  long long nacc = 0;
  for (int s = sl + tid; s < sh; s += kSegThreads) {  // the deferred replays' counts of these slots
    const long long v = D.nsw[s - lo];
    if (v) {
      nacc += v;
      D.nsw[s - lo] = 0;
    }
  }
  for (int lv = 0; lv < nlv; ++lv) {
    const int e0 = soff[g * nlv + lv] - eb, e1 = soff[g * nlv + lv + 1] - eb;
    for (int q = e0 + tid; q < e1; q += kSegThreads) {
      const int b = sE[q].b;
      const double lnb = sE[q].lnb;
      const int bl = b - clo, al = bl + 1;
      const double lb = cL[bl], la = cL[al];
      const double x = (lb - la) * cH[bl];  // (L[idx b] - L[idx a]) (T_b - T_a)/(T_b T_a), :803
      bool acc;
      const double dl = 1e-12 * (1.0 + fabs(lnb));
      if (lnb > -HUGE_VAL && x >= lnb + dl) acc = true;
      else if (lnb > -HUGE_VAL && x <= lnb - dl) acc = false;
      else acc = hbglibc::exp(x, T) >= betas[eb + q];
      if (acc) {
        const int ca = cC[al], cb = cC[bl];
        cL[al] = lb;
        cL[bl] = la;
        cC[al] = cb;
        cC[bl] = ca;
        if (b >= sl && b < sh) ++nacc;
      }
    }
    __syncthreads();
  }
  if (nacc) atomicAdd(&nacc_s, (unsigned long long)nacc);
  for (int s = sl + tid; s < sh; s += kSegThreads) D.idx_out[s] = cC[s - clo];
  if (iter % 100 == 0)
    for (int s = sl + tid; s < sh; s += kSegThreads) D.DEacc_arr[s - lo] = D.DEtrial_arr[s - lo] = 0;
  __syncthreads();
  if (tid == 0) {
    if (nacc_s) atomicAdd((unsigned long long*)&D.ctr->nswap, nacc_s);
    if (g == 0) swap_tail(D, iter, D.par, lo == 0 ? cC[0 - clo] : -1);
  }
}

// states and logL of the owned slots, by local slot (writer / verbose / download)
__global__ __launch_bounds__(kBlk) void ds_gather(Dev D, double* xs, double* ls, double* ps, int* oks) {
  const int j = blockIdx.x * kBlk + threadIdx.x;
  if (j >= D.nl) return;
  const int c = D.idx[D.lo + j];
  for (int i = 0; i < kNp; ++i) xs[(size_t)j * kNp + i] = D.x[(size_t)c * kNp + i];
  ls[j] = D.logL[c];
  if (ps) ps[j] = D.logP[c];
  if (oks) oks[j] = D.logP_ok[c];
}

// glibc-exact math on the device, for tests (fn 0 exp, 1 log, 2 pow, 3 sqrt, 4 div)
__global__ void ds_math_probe(int fn, const double* x, const double* y, long n, double* out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = x[i], b = y[i];
  out[i] = fn == 0 ? hbglibc::exp(a) : fn == 1 ? hbglibc::log(a) : fn == 2 ? hbglibc::pow(a, b)
         : fn == 3 ? sqrt(a) : a / b;
}

// Wall folds timed per wave, for diagnosis (scripts/wall_probe.py): lane i
// folds v[i] into [lo[i], hi[i]] (both walls reflecting); cyc[w]: the shader
// cycles wave w spent in hbwall::apply_wall.  One wave per workgroup.
__global__ void ds_wall_probe(const double* v, const double* lo, const double* hi, long n, double* out,
                              long long* cyc) {
  const long i = (long)blockIdx.x * 64 + (threadIdx.x & 63);
  const bool ok = i < n;
  const double x = ok ? v[i] : 0.0, l = ok ? lo[i] : 0.0, h = ok ? hi[i] : 1.0;
  long long t0, t1;
  __asm__ volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0) : "v"(x), "v"(l), "v"(h));
  const double y = hbwall::apply_wall(x, l, h, 1.0, 1.0);
  __asm__ volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(y));
  if (ok) out[i] = y;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x] = t1 - t0;
}

}  // namespace hbds

using namespace hbds;

#define DS_TRY(expr, what)                                   \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) {                                  \
      std::string m = std::string(what) + ": " + hipGetErrorString(_e); \
      return hbx_set_error(m.c_str());                       \
    }                                                        \
  } while (0)

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct hb_dsampler {
  hb_sampler* s = nullptr;
  hb_ctx* ctx = nullptr;
  hipStream_t st = nullptr;
  HbSamplerView v{};
  Params P{};
  Params* d_params = nullptr;
  Dev D{};
  int W = 0, NPAST = 0, device = 0;
  // sharding: owned slots [lo, lo + nl) of R ranks; m = largest shard,
  // nlmin = smallest (edge windows are capped at it)
  int lo = 0, nl = 0, R = 1, rank = 0, m = 0, nlmin = 0;
  // step_begin / all-gather / step_end: every sharded sampler, and a
  // one-rank one made by hb_dsampler_create_shard (the exchange path on a
  // single GPU: RCCL world size 1 in tests)
  bool xchg = false;
  std::vector<void*> allocs;
  std::vector<int> order;  // owned slots in descending temperature (ds_propose's wave order)
  // Swap schedules (SwapEnt | off | beta, compact), drawn ahead by producer
  // threads: the draws and levels of an iteration do not depend on any GPU
  // result, and hb_lagfib.hpp puts the glibc stream of iteration q at a known
  // offset (2 W q draws past the stream's state at creation), so the
  // schedules of several iterations are built in parallel, off the issuing
  // thread.  Iteration q uses ring slot q % R_RING: pinned -> copied into the
  // device slot by ds_propose (system-scope loads of the coldest waves).
  static constexpr int R_RING = 8;
  unsigned char* pin[R_RING] = {};
  unsigned char* d_sched[R_RING] = {};
  hipEvent_t ev_used[R_RING] = {};  // recorded after the swaps of every ev_every-th iteration (slot r)
  // an event after every swap launch costs a cache-flushing barrier packet
  // (~5 us of idle GPU before the next ds_propose, rocprof timeline); every
  // fourth iteration suffices for the producers' slot reuse
  static constexpr int ev_every = 4;  // divides R_RING: the events land on fixed ring slots
  long long q_issued = 0;  // iterations whose swaps are enqueued
  struct Slot {
    long long q = -1;       // iteration it holds (-1: never used)
    bool ready = false;     // schedule written
    bool released = false;  // its ds_swap_seg is enqueued and ev_used recorded
    bool overflow = false;  // more than kMaxLevels levels or sched_cap bytes: the step fails
    int nent = 0, nlv = 0;
    int maxent = 0;         // most attempts of one segment (ds_swap_seg stages them in LDS)
  };
  Slot slots[R_RING];
  std::mutex smu;
  std::condition_variable scv;
  std::vector<std::thread> workers;
  bool stop = false;
  // sticky failure: a producer could not reuse its ring slot, or an iteration
  // failed after its schedule was consumed (the device state is then partly
  // advanced): every later step / download returns this error (under smu)
  bool failed = false;
  std::string fail_msg;
  long long q_prod = 0, q_cons = 0, q_synced = 0;  // produced / consumed / skipped on the host stream
  uint32_t base_w[31] = {};                         // the swap stream at creation (hb_lagfib.hpp window)
  size_t sched_cap = 0;                             // bytes per ring slot
  int nthreads = 0;
  int nseg = 1;  // swap segments (ds_swap_seg workgroups) over the owned slots
  bool fused_prep = true;  // walker records in ds_propose's epilogue (else an hb_prep_kernel launch)
  double* d_lslot = nullptr; // [W] logL by slot after the Hastings test (one-process samplers)
  bool lslot_now = false;    // this iteration's fused Hastings test wrote d_lslot
  int* ecnt_buf[2] = {nullptr, nullptr};  // e-bin counters of even / odd iterations (Dev::ecnt)
  long long n_iter = 0;      // iterations begun (their parity: Dev::par, ecnt_buf)
  // Deferred swaps (one-process samplers on the ds_propose path): iteration
  // pend_iter's tempering swaps are replayed by the next ds_propose
  // (SwapPrev) instead of their own ds_swap_seg launch; ds_flush launches them
  // before anything reads the state (gather, download, sync, event drains).
  // HB_DS_DEFER=0 (A/B knob): never.
  bool defer = false;
  bool pend_on = false;
  int pend_slot = -1;
  long long pend_iter = -1;
  bool pend_lslot = false;
  int pend_par = 0;
  // a schedule the current iteration's ds_propose consumed (deferred swaps):
  // released in ds_end, after the likelihood launch, so the ring event (a
  // cache-flushing barrier packet) does not sit between ds_propose and it
  int rel_slot = -1;
  long long rel_q = -1;
  // host timers [s]: producer work (all threads), waits for a schedule, issue
  double t_prod = 0.0, t_wait = 0.0, t_issue = 0.0;
  // the iteration between step_begin and step_end
  int cur_slot = -1;
  long cur_iter = -1;
  long cur_n = 0;
  // staging for gathers / counters / events
  double* d_xs = nullptr;
  double* d_ls = nullptr;
  double* d_ps = nullptr;
  int* d_ok = nullptr;
  Counters* h_ctr = nullptr;
  Event* h_ev = nullptr;
  ~hb_dsampler() {
    {
      std::lock_guard<std::mutex> lk(smu);
      stop = true;
    }
    scv.notify_all();
    for (std::thread& t : workers) t.join();
    if (st) (void)hipStreamSynchronize(st);
    for (void* p : allocs) (void)hipFree(p);
    for (int r = 0; r < R_RING; ++r) {
      if (pin[r]) (void)hipHostFree(pin[r]);
      if (ev_used[r]) (void)hipEventDestroy(ev_used[r]);
    }
    if (h_ctr) (void)hipHostFree(h_ctr);
    if (h_ev) (void)hipHostFree(h_ev);
    if (st) (void)hipStreamDestroy(st);
  }
  template <class T>
  hipError_t alloc(T** p, size_t n) {
    hipError_t e = hipMalloc((void**)p, sizeof(T) * (n ? n : 1));
    if (e == hipSuccess) allocs.push_back((void*)*p);
    return e;
  }
};

static int ds_upload(hb_dsampler* d, const int* chain_of_slot);
static int ds_flush(hb_dsampler* d);

// Puts the sampler into its sticky failed state (first message wins) and
// wakes every waiter (producers and a ds_begin waiting for a schedule).
static void ds_mark_failed(hb_dsampler* d, const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(d->smu);
    if (!d->failed) {
      d->failed = true;
      d->fail_msg = msg;
    }
  }
  d->scv.notify_all();
}
// the failed state as an error return (0 if the sampler is healthy)
static int ds_check_failed(hb_dsampler* d, const char* where) {
  std::string m;
  {
    std::lock_guard<std::mutex> lk(d->smu);
    if (!d->failed) return 0;
    m = std::string(where) + ": the sampler failed earlier (" + d->fail_msg + "); destroy it";
  }
  return hbx_set_error(m.c_str());
}
// Marks the sampler failed unless disarmed: every return path of an iteration
// after its schedule was consumed (DS_TRY returns included).
struct DsFailGuard {
  hb_dsampler* d;
  bool armed = true;
  ~DsFailGuard() {
    if (armed) ds_mark_failed(d, std::string("an iteration failed after its schedule was consumed: ") + hb_last_error());
  }
};

// Builds iteration q's swap schedule into ring slot `slot`: the 2W draws of
// ptmcmc (:791, :810) from the stream jumped to 2 W q draws past creation,
// the dependency levels (attempt i follows every earlier attempt touching
// b_i or b_i + 1), and for each segment g of the owned slots the attempts
// whose pair lies in its cone [sl_g - nlv, sh_g + nlv) by level
// (ds_swap_seg).  Per-thread scratch in `sc`.
// the segments g of the owned slots [lo, lo + nl) whose cone
// [sl_g - nlv, sh_g + nlv) holds the pair (b, b + 1): sl_g - nlv <= b and
// b + 1 < sh_g + nlv, a contiguous range g0 .. g1 (empty: g0 > g1)
static void pair_segments(int b, int nlv, int lo, int nl, int G, int& g0, int& g1) {
  g0 = seg_of(b + 1 - nlv - lo, nl, G);
  while (g0 < G && seg_lo(lo, nl, g0 + 1, G) + nlv <= b + 1) ++g0;
  g1 = seg_of(b + nlv - lo, nl, G);
  while (g1 >= 0 && seg_lo(lo, nl, g1, G) - nlv > b) --g1;
}

// test hook (tests/test_dsampler.py): the producer's segment ranges
extern "C" int hbx_pair_segments(int b, int nlv, int lo, int nl, int G, int* g0, int* g1) {
  pair_segments(b, nlv, lo, nl, G, *g0, *g1);
  return 0;
}

struct SchedScratch {
  std::vector<int> b, lvl, last, cnt;
  std::vector<double> beta;
};
static void sched_build(hb_dsampler* d, long long q, int slot, SchedScratch& sc) {
  const int W = d->W, G = d->nseg, lo = d->lo, nl = d->nl;
  hb_dsampler::Slot& sl = d->slots[slot];
  sc.b.resize(W);
  sc.lvl.resize(W);
  sc.last.assign((size_t)W + 1, 0);
  sc.beta.resize(W);
  uint32_t w[31], c[31];
  memcpy(w, d->base_w, sizeof w);
  hblf::poly_xpow(2ull * (unsigned long long)W * (unsigned long long)q, c);
  hblf::window_jump(w, c);
  hblf::Stream gen(w);
  for (int i = 0; i < W; ++i) {  // ptmcmc :791, :810 (the expressions of hbx_swap_draws)
    sc.b[i] = (int)(((double)gen.rand() / (RAND_MAX)) * ((double)(W - 1)));
    sc.beta[i] = ((double)gen.rand() / (RAND_MAX));
  }
  int nlv = 0;
  for (int i = 0; i < W; ++i) {
    const int b = sc.b[i];
    if (b < 0 || b + 1 >= W) {  // rand() == RAND_MAX: the reference reads index[NCHAINS]; no swap here
      sc.lvl[i] = -1;
      continue;
    }
    const int l = std::max(sc.last[b], sc.last[b + 1]) + 1;
    sc.lvl[i] = l;
    sc.last[b] = sc.last[b + 1] = l;
    nlv = std::max(nlv, l);
  }
  sl.nlv = nlv;
  if (nlv > kMaxLevels) {
    sl.overflow = true;
    return;
  }
  // segments whose cone holds the pair (b, b + 1): sl_g - nlv <= b and
  // b + 1 < sh_g + nlv -- a contiguous range of g
  auto seg_range = [&](int b, int& g0, int& g1) { pair_segments(b, nlv, lo, nl, G, g0, g1); };
  sc.cnt.assign((size_t)G * nlv + 1, 0);
  size_t nent = 0;
  for (int i = 0; i < W; ++i) {
    if (sc.lvl[i] <= 0) continue;
    int g0, g1;
    seg_range(sc.b[i], g0, g1);
    for (int g = g0; g <= g1; ++g) {
      sc.cnt[(size_t)g * nlv + sc.lvl[i] - 1]++;
      ++nent;
    }
  }
  if (sched_bytes((size_t)G, (size_t)nlv, nent) > d->sched_cap) {
    sl.overflow = true;
    return;
  }
  unsigned char* buf = d->pin[slot];
  int* soff = reinterpret_cast<int*>(buf);
  SwapEnt* ent = reinterpret_cast<SwapEnt*>(buf + sched_ent_off((size_t)G, (size_t)nlv));
  double* betas = reinterpret_cast<double*>(buf + sched_beta_off((size_t)G, (size_t)nlv, nent));
  int run = 0;
  for (size_t k = 0; k < (size_t)G * nlv; ++k) {
    soff[k] = run;
    run += sc.cnt[k];
    sc.cnt[k] = soff[k];  // next free entry of (segment, level)
  }
  soff[(size_t)G * nlv] = run;
  int maxent = 0;
  for (int g = 0; g < G; ++g) maxent = std::max(maxent, soff[(size_t)(g + 1) * nlv] - soff[(size_t)g * nlv]);
  sl.maxent = maxent;
  for (int i = 0; i < W; ++i) {
    if (sc.lvl[i] <= 0) continue;
    int g0, g1;
    seg_range(sc.b[i], g0, g1);
    const double lnb = log(sc.beta[i]);
    for (int g = g0; g <= g1; ++g) {
      const int e = sc.cnt[(size_t)g * nlv + sc.lvl[i] - 1]++;
      ent[e].b = sc.b[i];
      ent[e].pad = 0;
      ent[e].lnb = lnb;
      betas[e] = sc.beta[i];
    }
  }
  sl.nent = (int)nent;
}

// producer thread: claims the next iteration, waits until its ring slot's
// previous schedule has been consumed (its ds_swap enqueued, then finished on
// the GPU), builds the schedule and publishes it
static void sched_worker(hb_dsampler* d) {
  (void)hipSetDevice(d->device);
  SchedScratch sc;
  constexpr int K = hb_dsampler::R_RING;
  while (true) {
    long long q;
    int slot, ev_slot = 0;
    bool reused;
    {
      std::unique_lock<std::mutex> lk(d->smu);
      d->scv.wait(lk, [&] {
        if (d->stop || d->failed) return true;
        const hb_dsampler::Slot& sl = d->slots[d->q_prod % K];
        if (sl.q < 0) return true;
        const long long q_rec = (sl.q / d->ev_every) * d->ev_every + d->ev_every - 1;  // next recorded event
        return sl.q == d->q_prod - K && sl.released && d->q_issued > q_rec;
      });
      if (d->stop || d->failed) return;
      q = d->q_prod++;
      slot = (int)(q % K);
      reused = d->slots[slot].q >= 0;
      if (reused) ev_slot = (int)(((d->slots[slot].q / d->ev_every) * d->ev_every + d->ev_every - 1) % K);
      d->slots[slot] = hb_dsampler::Slot{};
      d->slots[slot].q = q;
    }
    if (reused) {  // the GPU is done with the slot's previous schedule
      const hipError_t e = hipEventSynchronize(d->ev_used[ev_slot]);
      if (e != hipSuccess) {  // e.g. after a GPU fault: fail the sampler, do not leave ds_begin waiting
        ds_mark_failed(d, std::string("schedule producer: hipEventSynchronize: ") + hipGetErrorString(e));
        return;
      }
    }
    const double t0 = now_s();
    sched_build(d, q, slot, sc);
    const double dt = now_s() - t0;
    {
      std::lock_guard<std::mutex> lk(d->smu);
      d->slots[slot].ready = true;
      d->t_prod += dt;
    }
    d->scv.notify_all();
  }
}

// owned slots of rank r of R (hb_mcmc_amd/dist.py shard())
static inline int shard_lo(int W, int r, int R) { return (int)((long long)W * r / R); }

static hb_dsampler* ds_create(hb_sampler* s, hb_ctx* ctx, const int* chain_of_slot, int R, int rank) {
  if (!s || !ctx) {
    hbx_set_error("hb_dsampler_create: null sampler or context");
    return nullptr;
  }
  hb_dsampler* d = new hb_dsampler();
  d->s = s;
  d->ctx = ctx;
  hbx_sampler_view(s, &d->v);
  const HbSamplerView& v = d->v;
  if (R < 1 || rank < 0 || rank >= R || v.W < 2 * R) {
    hbx_set_error("hb_dsampler_create: bad rank / rank count (every rank needs two slots)");
    delete d;
    return nullptr;
  }
  if (v.lo != shard_lo(v.W, rank, R) || v.hi != shard_lo(v.W, rank + 1, R)) {
    hbx_set_error(R == 1 ? "hb_dsampler_create: the sampler must own every slot (one GPU)"
                         : "hb_dsampler_create_shard: the sampler must own slots [W r/R, W (r+1)/R)");
    delete d;
    return nullptr;
  }
  d->W = v.W;
  d->NPAST = v.NPAST;
  d->R = R;
  d->rank = rank;
  d->xchg = chain_of_slot != nullptr;
  d->lo = v.lo;
  d->nl = v.hi - v.lo;
  d->m = 0;
  d->nlmin = v.W;
  for (int r = 0; r < R; ++r) {
    const int n = shard_lo(v.W, r + 1, R) - shard_lo(v.W, r, R);
    d->m = std::max(d->m, n);
    d->nlmin = std::min(d->nlmin, n);
  }
  d->device = hbx_ctx_device(ctx);
  if (hb_reserve(ctx, d->nl)) {  // the likelihood workspace, before anything is enqueued
    delete d;
    return nullptr;
  }
  auto fail = [&](const char* what, hipError_t e) -> hb_dsampler* {
    std::string m = std::string("hb_dsampler_create: ") + what + ": " + hipGetErrorString(e);
    hbx_set_error(m.c_str());
    delete d;
    return nullptr;
  };
  hipError_t e = hipSetDevice(d->device);
  if (e != hipSuccess) return fail("hipSetDevice", e);
  if ((e = hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
  const int W = d->W;
  const size_t Wz = (size_t)W, Nz = (size_t)d->nl;
  Dev& D = d->D;
  D.lo = d->lo;
  D.nl = d->nl;
  // by chain / ladder: W entries; by slot: the nl owned slots
  if ((e = d->alloc(&D.x, Wz * kNp)) || (e = d->alloc(&D.logL, Wz)) || (e = d->alloc(&D.logP, Wz)) ||
      (e = d->alloc(&D.logP_ok, Wz)) || (e = d->alloc(&D.idx, Wz)) || (e = d->alloc(&D.idx_out, Wz)) || (e = d->alloc(&D.order, Nz)) ||

      (e = d->alloc(&D.temp, Wz)) || (e = d->alloc(&D.idum, Nz)) || (e = d->alloc(&D.idum2, Nz)) ||
      (e = d->alloc(&D.iy, Nz)) || (e = d->alloc(&D.iset, Nz)) || (e = d->alloc(&D.gset, Nz)) ||
      (e = d->alloc(&D.cts, Nz)) || (e = d->alloc(&D.iv, Nz * NTAB)) || (e = d->alloc(&D.y, Nz * kNp)) ||
      (e = d->alloc(&D.logPy, Nz)) || (e = d->alloc(&D.alpha2, Nz)) || (e = d->alloc(&D.logLy, Nz)) ||
      (e = d->alloc(&D.jump, Nz)) || (e = d->alloc(&D.jtype, Nz)) ||
      (e = d->alloc(&D.hist, Nz * (size_t)d->NPAST * kNp)) || (e = d->alloc(&D.DEacc_arr, Nz)) ||
      (e = d->alloc(&D.DEtrial_arr, Nz)) || (e = d->alloc(&D.nsw, Nz)) || (e = d->alloc(&D.ctr, 1)) || (e = d->alloc(&D.ev, (size_t)kEvCap)) ||
      (e = d->alloc(&d->d_xs, Nz * kNp)) || (e = d->alloc(&d->d_ls, Nz)) || (e = d->alloc(&d->d_ps, Nz)) ||
      (e = d->alloc(&d->d_ok, Nz)) || (e = d->alloc(&D.hs, Wz)) || (e = d->alloc(&d->d_params, 1)))
    return fail("hipMalloc", e);
  D.P = d->d_params;
  if ((e = hipMemsetAsync(D.nsw, 0, sizeof(long long) * Nz, d->st))) return fail("hipMemset", e);
  // eval order by e bins (AccArgs::ecnt) up to kEvalOrdMax owned slots
  if (Nz <= (size_t)kEvalOrdMax) {
    if ((e = d->alloc(&D.ecnt, 2 * (size_t)kOrdBins * kEbinStride)) || (e = d->alloc(&D.elist, (size_t)kOrdBins * Nz)))
      return fail("hipMalloc", e);
    if ((e = hipMemsetAsync(D.ecnt, 0, 2 * sizeof(int) * kOrdBins * kEbinStride, d->st))) return fail("hipMemset", e);
    d->ecnt_buf[0] = D.ecnt;
    d->ecnt_buf[1] = D.ecnt + (size_t)kOrdBins * kEbinStride;
    D.ecnt_next = d->ecnt_buf[1];
  }
  // records in ds_propose's epilogue while the slots fit one resident round
  // of its waves at that occupancy (4 per SIMD, 16 per CU)
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d->device) != hipSuccess || cus <= 0)
      cus = 256;
    d->fused_prep = d->nl <= 16 * cus;
  }
  // swap segments of <= kSegSlots owned slots; an attempt is listed for at
  // most min(G, 3 + 2 kMaxLevels / (smallest segment)) segments
  d->nseg = std::max(1, (d->nl + kSegSlots - 1) / kSegSlots);
  {
    const bool one = !d->xchg && d->lo == 0 && d->nl == W;
    if (one && (e = d->alloc(&d->d_lslot, Wz))) return fail("hipMalloc", e);
    const char* df = getenv("HB_DS_DEFER");
    d->defer = one && (df ? atoi(df) != 0 : true);
  }
  {
    const size_t G = (size_t)d->nseg, segmin = std::max<size_t>(1, (size_t)d->nl / G);
    const size_t per = std::min(G, 3 + 2 * (size_t)kMaxLevels / segmin);
    d->sched_cap = sched_bytes(G, (size_t)kMaxLevels, Wz * per);
  }
  for (int r = 0; r < hb_dsampler::R_RING; ++r) {
    if ((e = d->alloc(&d->d_sched[r], d->sched_cap))) return fail("hipMalloc", e);
    if ((e = hipHostMalloc((void**)&d->pin[r], d->sched_cap, hipHostMallocDefault))) return fail("pinned", e);
    // the event only tells the producer that the GPU has finished reading the
    // slot (ds_propose's pinned-source loads): no system-scope release is
    // needed for that, and without it the barrier packet writes back and
    // invalidates no caches before the next launch (with the fence: within
    // noise, profiles/r05/r05v_ds_event_fence_ab.txt)
    if ((e = hipEventCreateWithFlags(&d->ev_used[r], hipEventDisableTiming | hipEventDisableSystemFence)))
      return fail("event", e);
  }
  if ((e = hipHostMalloc((void**)&d->h_ctr, sizeof(Counters), hipHostMallocDefault))) return fail("pinned", e);
  if ((e = hipHostMalloc((void**)&d->h_ev, sizeof(Event) * kEvCap, hipHostMallocDefault))) return fail("pinned", e);
  Params& P = d->P;
  P.W = W;
  P.NPAST = d->NPAST;
  P.log_on = v.log != nullptr;
  P.log_lc_period = v.log_lc_period;
  P.LC_PERIOD = v.LC_PERIOD;
  for (int i = 0; i < kNp; ++i) {
    P.lim_lo[i] = v.limits[i].lo;
    P.lim_hi[i] = v.limits[i].hi;
    P.fl_lo[i] = v.limited[i].lo;
    P.fl_hi[i] = v.limited[i].hi;
    P.sigma_p[i] = v.sigma_p[i];
    P.gpflag[i] = v.gp[i].flag;
  }
  if (ds_upload(d, chain_of_slot)) {
    delete d;
    return nullptr;
  }
  // schedule producers: the swap stream as it stands now is iteration 0's start
  if (hbx_swap_rng_window(s, d->base_w)) return fail("swap stream", hipErrorInvalidValue);
  const char* nt = getenv("HB_DS_SCHED_THREADS");
  // 4 producers: with 2 (the default until round 6) one schedule took about
  // as long as one GPU iteration (154 us of building per iteration over both
  // threads at W = 4096, bench.py device_loop.host_us_per_iter), so a slower
  // host stalled the loop; 8 brought one 0.118-ms run on the box's 16-core
  // share (profiles/r06/r06zn_ds_threads_ab.txt, r06zo_ds_threads_ab.txt)
  d->nthreads = nt ? std::max(1, atoi(nt)) : 4;
  for (int i = 0; i < d->nthreads; ++i) d->workers.emplace_back(sched_worker, d);
  return d;
}

extern "C" hb_dsampler* hb_dsampler_create(hb_sampler* s, hb_ctx* ctx) { return ds_create(s, ctx, nullptr, 1, 0); }

extern "C" hb_dsampler* hb_dsampler_create_shard(hb_sampler* s, hb_ctx* ctx, const int* chain_of_slot, int nranks,
                                                 int rank) {
  if (!chain_of_slot) {
    hbx_set_error("hb_dsampler_create_shard: chain_of_slot is required");
    return nullptr;
  }
  return ds_create(s, ctx, chain_of_slot, nranks, rank);
}

// A deferred tempering swap still pending here (pend_on) is dropped on
// purpose: the device state goes with the sampler.  Every entry point that
// READS the state (download, gather, sync, init_logl, the event drain) calls
// ds_flush first; a new reader must do the same.
extern "C" void hb_dsampler_destroy(hb_dsampler* d) { delete d; }

// host sampler (owned slots, by slot) -> device (by chain); chain_of_slot
// (all W slots) may be NULL when the sampler owns every slot
static int ds_upload(hb_dsampler* d, const int* chain_of_slot) {
  const HbSamplerView& v = d->v;
  const int W = d->W, lo = d->lo, nl = d->nl;
  const size_t Wz = (size_t)W, Nz = (size_t)nl;
  Dev& D = d->D;
  std::vector<double> x(Wz * kNp, 0.0), L(Wz, 0.0), Pp(Wz, 0.0), gset(Nz);
  std::vector<int> ok(Wz, 0), idx(Wz), idum(Nz), idum2(Nz), iy(Nz), iset(Nz), iv(Nz * NTAB);
  std::vector<long long> cts(Nz);
  std::vector<char> seen(Wz, 0);
  for (int j = 0; j < W; ++j) {
    const int c = chain_of_slot ? chain_of_slot[j] : v.cid[j];
    if (c < 0 || c >= W || seen[c]) return hbx_set_error("hb_dsampler: chain_of_slot is not a permutation");
    seen[c] = 1;
    idx[j] = c;
  }
  for (int jl = 0; jl < nl; ++jl) {
    const int c = v.cid[jl];
    if (idx[lo + jl] != c) return hbx_set_error("hb_dsampler: chain_of_slot disagrees with the sampler's slots");
    memcpy(&x[(size_t)c * kNp], &v.x[(size_t)jl * kNp], sizeof(double) * kNp);
    L[c] = v.logL[jl];
    Pp[c] = v.logP[jl];
    ok[c] = v.logP_ok[jl] ? 1 : 0;
    const RNG_Vars& r = v.states[jl];
    if (v.seeds[jl] > 2147483647L || v.seeds[jl] < -2147483647L) return hbx_set_error("hb_dsampler: seed out of range");
    idum[jl] = (int)v.seeds[jl];
    idum2[jl] = (int)r.idum2;
    iy[jl] = (int)r.iy;
    iset[jl] = r.iset;
    gset[jl] = r.gset;
    cts[jl] = r.cts;
    for (int t = 0; t < NTAB; ++t) iv[(size_t)jl * NTAB + t] = (int)r.iv[t];
  }
  Counters c{};
  c.acc = *v.acc;
  c.DEacc = *v.DEacc;
  c.DEtrial = *v.DEtrial;
  c.atrial = *v.atrial;
  c.cold_acc = *v.cold_acc;
  c.nswap = *v.nswap;
  for (int jl = 0; jl < nl; ++jl) {
    c.DEacc_tot += v.DEacc_arr[jl];
    c.DEtrial_tot += v.DEtrial_arr[jl];
    c.acc_it += v.acc_arr[jl];
  }
  c.logLmap = -1.0 / 0.0;
  hipStream_t s = d->st;
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  DS_TRY(hipMemcpyAsync(D.x, x.data(), sizeof(double) * x.size(), hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.logL, L.data(), sizeof(double) * Wz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.logP, Pp.data(), sizeof(double) * Wz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.logP_ok, ok.data(), sizeof(int) * Wz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.idx, idx.data(), sizeof(int) * Wz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.idx_out, idx.data(), sizeof(int) * Wz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.temp, v.temp, sizeof(double) * Wz, hipMemcpyHostToDevice, s), "upload");
  // propose waves in descending temperature: the hot rungs' long wall runs
  // are dispatched first (ds_propose lasts as long as its latest-finishing
  // wave), kPW consecutive ones per workgroup
  d->order.resize(Nz);
  for (size_t i = 0; i < Nz; ++i) d->order[i] = lo + (int)i;
  std::stable_sort(d->order.begin(), d->order.end(), [&](int a, int b) { return v.temp[a] > v.temp[b]; });
  DS_TRY(hipMemcpyAsync(D.order, d->order.data(), sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  std::vector<double> hs(Wz, 0.0);
  for (int b = 0; b + 1 < W; ++b) {  // ptmcmc's H (:803) for the pair (a, b) = (b+1, b): same IEEE ops
    const double heat1 = v.temp[b + 1], heat2 = v.temp[b];
    hs[b] = (heat2 - heat1) / (heat2 * heat1);
  }
  DS_TRY(hipMemcpyAsync(D.hs, hs.data(), sizeof(double) * Wz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(d->d_params, &d->P, sizeof(Params), hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.idum, idum.data(), sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.idum2, idum2.data(), sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.iy, iy.data(), sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.iset, iset.data(), sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.gset, gset.data(), sizeof(double) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.cts, cts.data(), sizeof(long long) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.iv, iv.data(), sizeof(int) * iv.size(), hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.hist, v.hist, sizeof(double) * Nz * d->NPAST * kNp, hipMemcpyHostToDevice, s),
         "upload");
  DS_TRY(hipMemcpyAsync(D.DEacc_arr, v.DEacc_arr, sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.DEtrial_arr, v.DEtrial_arr, sizeof(int) * Nz, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipMemcpyAsync(D.ctr, &c, sizeof c, hipMemcpyHostToDevice, s), "upload");
  DS_TRY(hipStreamSynchronize(s), "upload sync");
  return 0;
}

// device -> host sampler (owned slots, by slot); also drains the big-jump records
static int ds_drain_events(hb_dsampler* d);

extern "C" int hb_dsampler_download(hb_dsampler* d) {
  if (!d) return hbx_set_error("hb_dsampler_download: null");
  if (const int rc = ds_check_failed(d, "hb_dsampler_download")) return rc;
  if (const int rc = ds_flush(d)) return rc;
  const HbSamplerView& v = d->v;
  const int nl = d->nl;
  const size_t Nz = (size_t)nl;
  Dev& D = d->D;
  hipStream_t s = d->st;
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  ds_gather<<<(nl + kBlk - 1) / kBlk, kBlk, 0, s>>>(D, d->d_xs, d->d_ls, d->d_ps, d->d_ok);
  DS_TRY(hipGetLastError(), "gather");
  std::vector<int> idx(Nz), ok(Nz), idum(Nz), idum2(Nz), iy(Nz), iset(Nz), iv(Nz * NTAB);
  std::vector<double> gset(Nz);
  std::vector<long long> cts(Nz);
  DS_TRY(hipMemcpyAsync(v.x, d->d_xs, sizeof(double) * Nz * kNp, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(v.logL, d->d_ls, sizeof(double) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(v.logP, d->d_ps, sizeof(double) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(ok.data(), d->d_ok, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(idx.data(), D.idx + d->lo, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(idum.data(), D.idum, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(idum2.data(), D.idum2, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(iy.data(), D.iy, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(iset.data(), D.iset, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(gset.data(), D.gset, sizeof(double) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(cts.data(), D.cts, sizeof(long long) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(iv.data(), D.iv, sizeof(int) * iv.size(), hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(v.hist, D.hist, sizeof(double) * Nz * d->NPAST * kNp, hipMemcpyDeviceToHost, s),
         "download");
  DS_TRY(hipMemcpyAsync(v.DEacc_arr, D.DEacc_arr, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(v.DEtrial_arr, D.DEtrial_arr, sizeof(int) * Nz, hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipMemcpyAsync(d->h_ctr, D.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s), "download");
  DS_TRY(hipStreamSynchronize(s), "download sync");
  for (int j = 0; j < nl; ++j) {
    v.cid[j] = idx[j];
    v.logP_ok[j] = (char)ok[j];
    v.seeds[j] = idum[j];
    RNG_Vars& r = v.states[j];
    r.idum2 = idum2[j];
    r.iy = iy[j];
    r.iset = iset[j];
    r.gset = gset[j];
    r.cts = cts[j];
    for (int t = 0; t < NTAB; ++t) r.iv[t] = iv[(size_t)j * NTAB + t];
    v.acc_arr[j] = 0;  // cleared by every accept step (hb_sampler_accept)
  }
  const Counters& c = *d->h_ctr;
  *v.acc = c.acc;
  *v.DEacc = c.DEacc;
  *v.DEtrial = c.DEtrial;
  *v.atrial = c.atrial;
  *v.cold_acc = c.cold_acc;
  *v.nswap = c.nswap;
  // the host's swap stream: the draws of the iterations run on the device
  // since the last download (two per attempt, W attempts each)
  if (d->q_cons > d->q_synced) {
    if (hbx_swap_rng_skip(d->s, 2ull * (unsigned long long)d->W * (unsigned long long)(d->q_cons - d->q_synced)))
      return hbx_set_error("hb_dsampler_download: swap stream");
    d->q_synced = d->q_cons;
  }
  return ds_drain_events(d);
}

static int ds_drain_events(hb_dsampler* d) {
  if (const int rc = ds_flush(d)) return rc;
  DS_TRY(hipMemcpyAsync(d->h_ctr, d->D.ctr, sizeof(Counters), hipMemcpyDeviceToHost, d->st), "events");
  DS_TRY(hipStreamSynchronize(d->st), "events");
  const int n = std::min(d->h_ctr->nev, kEvCap);
  if (d->h_ctr->nev > kEvCap) return hbx_set_error("hb_dsampler: big-jump record buffer overflowed");
  if (n == 0) return 0;
  DS_TRY(hipMemcpyAsync(d->h_ev, d->D.ev, sizeof(Event) * n, hipMemcpyDeviceToHost, d->st), "events");
  const int zero = 0;
  DS_TRY(hipMemcpyAsync(&d->D.ctr->nev, &zero, sizeof(int), hipMemcpyHostToDevice, d->st), "events");
  DS_TRY(hipStreamSynchronize(d->st), "events");
  std::vector<Event> evs(d->h_ev, d->h_ev + n);
  // the host sampler logs in slot order within an iteration (slots 0..5)
  std::stable_sort(evs.begin(), evs.end(), [](const Event& a, const Event& b) {
    return a.iter != b.iter ? a.iter < b.iter : a.slot < b.slot;
  });
  for (const Event& e : evs)
    hbx_log_big_jump(d->v.log, (long)e.iter, e.chain, e.H, e.alpha, e.tmp, e.lx, e.ly, e.px, e.py, e.xo, e.xn,
                     e.jtype);
  return 0;
}

namespace hbds {
// MAP tracker seeded with the chain in slot 0
__global__ void ds_seed_map(Dev D) {
  const int c0 = D.idx[0];
  if (threadIdx.x < kNp) D.ctr->xmap[threadIdx.x] = D.x[(size_t)c0 * kNp + threadIdx.x];
  if (threadIdx.x == 0) D.ctr->logLmap = D.logL[c0];
}
// logL[chain of owned slot j] = ls[j]
__global__ __launch_bounds__(kBlk) void ds_scatter_logl(Dev D, const double* __restrict__ ls) {
  const int j = blockIdx.x * kBlk + threadIdx.x;
  if (j < D.nl) D.logL[D.idx[D.lo + j]] = ls[j];
}
}  // namespace hbds

// iteration-0 recompute (:488): logL of every current state, and the MAP
// tracker seeded with chain 0's state (:342; the rank owning chain 0)
extern "C" int hb_dsampler_init_logl(hb_dsampler* d) {
  if (!d) return hbx_set_error("hb_dsampler_init_logl: null");
  if (const int rc = ds_flush(d)) return rc;
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  if (d->R == 1) {
    const int rc = hb_loglik_batch_dev(d->ctx, d->D.x, d->W, d->D.logL, (void*)d->st);
    if (rc) return rc;
  } else {  // owned slots only: states by slot -> likelihood -> logL by chain
    ds_gather<<<(d->nl + kBlk - 1) / kBlk, kBlk, 0, d->st>>>(d->D, d->d_xs, d->d_ls, nullptr, nullptr);
    DS_TRY(hipGetLastError(), "gather");
    const int rc = hb_loglik_batch_dev(d->ctx, d->d_xs, d->nl, d->d_ls, (void*)d->st);
    if (rc) return rc;
    ds_scatter_logl<<<(d->nl + kBlk - 1) / kBlk, kBlk, 0, d->st>>>(d->D, d->d_ls);
    DS_TRY(hipGetLastError(), "scatter");
  }
  // logLmap / xmap of the chain in slot 0 (chain 0 at the reference's start,
  // :342; the rank owning slot 0 computed its logL above, whatever the
  // chain_of_slot permutation of an advanced state)
  ds_seed_map<<<1, 64, 0, d->st>>>(d->D);
  DS_TRY(hipGetLastError(), "map");
  return 0;
}

extern "C" long hb_dsampler_exchange_cap(const hb_dsampler* d) {
  if (!d) return hbx_set_error("hb_dsampler_exchange_cap: null");
  return (long)d->m + 2L * d->nlmin * kRec;
}

extern "C" void* hb_dsampler_stream(hb_dsampler* d) { return d ? (void*)d->st : nullptr; }

extern "C" int hb_dsampler_host_times(const hb_dsampler* d, double* out4) {
  if (!d || !out4) return hbx_set_error("hb_dsampler_host_times: null");
  hb_dsampler* m = const_cast<hb_dsampler*>(d);
  std::lock_guard<std::mutex> lk(m->smu);
  out4[0] = d->t_prod;
  out4[1] = d->t_wait;
  out4[2] = d->t_issue;
  out4[3] = d->nthreads;
  return 0;
}

// first half of an iteration: the iteration's swap schedule (a producer
// thread built it into the pinned ring), proposals, likelihood + Hastings
// test of the owned slots; exchanging samplers also pack the rank's
// all-gather contribution into send
// Iteration q's schedule (ring slot `slot`) is consumed by a launch now on the
// sampler's stream: its producer may reuse the slot once the next recorded
// event has completed.
static int ds_release(hb_dsampler* d, int slot, long long q) {
  if ((q + 1) % d->ev_every == 0) DS_TRY(hipEventRecord(d->ev_used[slot], d->st), "schedule ring");
  {
    std::lock_guard<std::mutex> lk(d->smu);
    d->slots[slot].released = true;
    d->q_issued = q + 1;
  }
  d->scv.notify_all();
  return 0;
}
// iteration `iter`'s tempering swaps and bookkeeping by ds_swap_seg (its
// schedule in ring slot `slot`, `par` its parity); X: the all-gather of an
// exchanging sampler (null: one process, logL by slot from d_lslot when lslot)
static int ds_swap_launch(hb_dsampler* d, int slot, long long iter, bool lslot, int par, const Gathered* X) {
  const hb_dsampler::Slot sl = d->slots[slot];  // written by its producer before the ready flag
  const int G = d->nseg;
  const unsigned char* base = d->d_sched[slot];
  const int* d_soff = reinterpret_cast<const int*>(base);
  const SwapEnt* d_ent = reinterpret_cast<const SwapEnt*>(base + sched_ent_off((size_t)G, (size_t)sl.nlv));
  const double* d_beta =
      reinterpret_cast<const double*>(base + sched_beta_off((size_t)G, (size_t)sl.nlv, (size_t)sl.nent));
  // LDS: the widest cone's (logL, chain, pair factor) and the largest
  // segment's attempts
  const size_t wc_max = (size_t)(d->nl + G - 1) / G + 2 * (size_t)sl.nlv;
  const size_t lds = sizeof(SwapEnt) * (size_t)sl.maxent + (2 * sizeof(double) + sizeof(int)) * wc_max;
  Dev Dx = d->D;
  Dx.par = par;
  if (X) {
    ds_swap_seg<true><<<G, kSegThreads, lds, d->st>>>(Dx, d->W, d_soff, d_ent, d_beta, sl.nlv, G, iter, *X, nullptr);
  } else {
    const Gathered none{nullptr, 0, 1, 0, 0, 0};
    ds_swap_seg<false><<<G, kSegThreads, lds, d->st>>>(Dx, d->W, d_soff, d_ent, d_beta, sl.nlv, G, iter, none,
                                                       lslot ? d->d_lslot : nullptr);
  }
  DS_TRY(hipGetLastError(), "ds_swap_seg");
  return 0;
}
// the deferred swaps of the last iteration by their own launch (before
// anything reads the sampler's state)
static int ds_flush(hb_dsampler* d) {
  if (!d->pend_on) return 0;
  d->pend_on = false;
  DsFailGuard guard{d};
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  if (const int rc = ds_swap_launch(d, d->pend_slot, d->pend_iter, d->pend_lslot, d->pend_par, nullptr)) return rc;
  std::swap(d->D.idx, d->D.idx_out);
  if (const int rc = ds_release(d, d->pend_slot, d->pend_iter)) return rc;
  guard.armed = false;
  return 0;
}
// per-wave LDS of the deferred swaps' replay in ds_propose, at most
constexpr size_t kSwapPrevLdsMax = 32768;

static long ds_begin(hb_dsampler* d, long iter, double* send, long cap) {
  const int W = d->W;
  const Dev& D = d->D;
  hipStream_t s = d->st;
  if (d->cur_iter >= 0) return hbx_set_error("hb_dsampler: step_begin twice without step_end");
  if (const int rc = ds_check_failed(d, "hb_dsampler_step")) return rc;
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  const double tw0 = now_s();
  const long long q = d->q_cons;
  const int slot = (int)(q % hb_dsampler::R_RING);
  hb_dsampler::Slot sl;
  {
    std::unique_lock<std::mutex> lk(d->smu);
    d->scv.wait(lk, [&] { return d->failed || (d->slots[slot].q == q && d->slots[slot].ready); });
    sl = d->slots[slot];
  }
  if (const int rc = ds_check_failed(d, "hb_dsampler_step")) return rc;  // a producer failed
  // from here on the iteration's schedule is consumed: any failure leaves the
  // device state partly advanced, so it is sticky (DsFailGuard); q_cons
  // advances only when the iteration's swaps are enqueued (ds_end)
  DsFailGuard guard{d};
  const double tw1 = now_s();
  if (sl.overflow)
    return hbx_set_error("hb_dsampler: an iteration's swap schedule exceeds its buffer (more than 64 levels)");
  const size_t used_bytes = sched_bytes((size_t)d->nseg, (size_t)sl.nlv, (size_t)sl.nent);  // a multiple of 8
  const int NPAST = d->NPAST, nl = d->nl;
  // the iteration's parity: its e-bin counters and DE-trial slot
  {
    const int par = (int)(d->n_iter & 1);
    d->D.par = par;
    if (d->ecnt_buf[0]) {
      d->D.ecnt = d->ecnt_buf[par];
      d->D.ecnt_next = d->ecnt_buf[par ^ 1];
    }
    d->n_iter++;
  }
  // the previous iteration's deferred swaps: replayed by this ds_propose when
  // their per-wave scratch fits, else by their own launch first
  SwapPrev SP{};
  size_t sp_lds = 0;
  bool fuse = false;
  if (d->pend_on) {
    const hb_dsampler::Slot& ps = d->slots[d->pend_slot];
    const int cone = 2 * ps.nlv + 1;
    sp_lds = (size_t)kPW * swap_prev_wave_bytes(cone, ps.maxent);
    if (sp_lds <= kSwapPrevLdsMax) {
      const int G = d->nseg;
      const unsigned char* base = d->d_sched[d->pend_slot];
      SP.soff = reinterpret_cast<const int*>(base);
      SP.ent = reinterpret_cast<const SwapEnt*>(base + sched_ent_off((size_t)G, (size_t)ps.nlv));
      SP.betas = reinterpret_cast<const double*>(base + sched_beta_off((size_t)G, (size_t)ps.nlv, (size_t)ps.nent));
      SP.Ls = d->pend_lslot ? d->d_lslot : nullptr;
      SP.idx_out = D.idx_out;
      SP.iter = d->pend_iter;
      SP.nlv = ps.nlv;
      SP.G = G;
      SP.cone = cone;
      SP.maxent = ps.maxent;
      fuse = true;
    } else if (const int rc = ds_flush(d)) {
      return rc;
    }
  }
  // proposals, and in their epilogue the likelihood's walker records (the
  // context's workspace, looked up per launch: another caller may have grown it)
  Dev Dp = D;
  {
    void* wc = nullptr;
    double* tab_pc = nullptr;
    const int rc = hbx_ctx_prep_args(d->ctx, &wc, &Dp.ma, &tab_pc);
    if (rc) return rc;
    Dp.wc = static_cast<double*>(wc);
    Dp.tab_pc = tab_pc;
  }
  auto* sch_src = reinterpret_cast<const unsigned long long*>(d->pin[slot]);
  auto* sch_dst = reinterpret_cast<unsigned long long*>(d->d_sched[slot]);
  const long long n8 = (long long)(used_bytes / 8);
  {
    const unsigned pg = (unsigned)((nl + kPW - 1) / kPW);
    if (fuse) {
      Dp.idx = D.idx;  // the previous iteration's index[] (the replay's input)
      if (d->fused_prep)
        ds_propose<true, true><<<pg, 64 * kPW, sp_lds, s>>>(Dp, W, NPAST, (long long)iter, sch_src, sch_dst, n8, SP);
      else
        ds_propose<false, true><<<pg, 64 * kPW, sp_lds, s>>>(Dp, W, NPAST, (long long)iter, sch_src, sch_dst, n8, SP);
    } else if (d->fused_prep) {
      ds_propose<true, false><<<pg, 64 * kPW, 0, s>>>(Dp, W, NPAST, (long long)iter, sch_src, sch_dst, n8, SwapPrev{});
    } else {
      ds_propose<false, false><<<pg, 64 * kPW, 0, s>>>(Dp, W, NPAST, (long long)iter, sch_src, sch_dst, n8, SwapPrev{});
    }
    DS_TRY(hipGetLastError(), "ds_propose");
    if (fuse) {  // this iteration reads the index[] the replay wrote; the schedule is consumed
      d->pend_on = false;
      std::swap(d->D.idx, d->D.idx_out);
      d->rel_slot = d->pend_slot;
      d->rel_q = d->pend_iter;
    }
    if (!d->fused_prep) {
      const int rc = hb_prepare_dev(d->ctx, D.y, nl, (void*)s);
      if (rc) return rc;
    }
    // likelihood with the Hastings test fused into its waves' epilogue
    // (hb_accept.hpp); ds_accept only where the plan has no one-wave kernel
    AccArgs acc{D.idx, D.logL, D.logP, D.logPy, D.temp, D.alpha2, D.jump, D.jtype, D.x, D.y, D.hist,
                D.DEacc_arr, D.ctr, D.ev, d->P.log_on, NPAST, (long long)iter, d->lo, 0,
                D.ecnt, D.elist, nl, 0, d->d_lslot, D.ecnt_next};  // Lslot: null for exchanging samplers
    int rc = hbx_loglik_accept_dev(d->ctx, D.y, nl, D.logLy, &acc, (void*)s);
    d->lslot_now = rc == 0 && acc.Lslot != nullptr;
    if (rc == 1) {
      rc = hb_evaluate_dev(d->ctx, nl, D.logLy, 0, (void*)s);
      if (rc) return rc;
      ds_accept<<<(nl + 63) / 64, kAccThreads, 0, s>>>(D, W, NPAST, (long long)iter);
      DS_TRY(hipGetLastError(), "ds_accept");
    } else if (rc) {
      return rc;
    }
  }
  long n = 0;
  if (d->xchg) {
    const int ke = std::min(sl.nlv, d->nlmin);  // edge window (a level moves a chain by one slot)
    n = (long)d->m + 2L * ke * kRec;
    if (!send || n > cap) return hbx_set_error("hb_dsampler_step_begin: send buffer missing or too small");
    const long thr = n;
    ds_pack<<<(unsigned)((thr + kPackThreads - 1) / kPackThreads), kPackThreads, 0, s>>>(D, send, d->m, ke);
    DS_TRY(hipGetLastError(), "ds_pack");
  }
  d->cur_slot = slot;
  d->cur_iter = iter;
  d->cur_n = n;
  d->t_wait += tw1 - tw0;
  d->t_issue += now_s() - tw1;
  guard.armed = false;
  return n;
}

// second half: import the all-gather (exchanging samplers), tempering swaps,
// bookkeeping
static int ds_end(hb_dsampler* d, long iter, const double* recv, long n) {
  if (const int rc = ds_check_failed(d, "hb_dsampler_step_end")) return rc;
  if (d->cur_iter != iter) return hbx_set_error("hb_dsampler_step_end: no step_begin for this iteration");
  // a caller mistake is recoverable (step_end may be called again with the
  // right buffer): checked before the guard is armed
  if (d->xchg && (!recv || n != d->cur_n))
    return hbx_set_error("hb_dsampler_step_end: gathered buffer missing or of the wrong size");
  // the iteration's proposals and likelihood are enqueued: failing from here
  // on is sticky, like the second half of ds_begin
  DsFailGuard guard{d};
  const double t0 = now_s();
  const int slot = d->cur_slot;
  const hb_dsampler::Slot sl = d->slots[slot];  // written by its producer before the ready flag
  d->cur_iter = -1;
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  if (d->rel_slot >= 0) {  // the previous iteration's schedule, consumed by this ds_propose
    const int rs = d->rel_slot;
    d->rel_slot = -1;
    if (const int rc = ds_release(d, rs, d->rel_q)) return rc;
  }
  if (d->defer && !d->xchg) {
    // the swaps wait for the next ds_propose (SwapPrev) or ds_flush
    d->pend_on = true;
    d->pend_slot = slot;
    d->pend_iter = iter;
    d->pend_lslot = d->lslot_now;
    d->pend_par = d->D.par;
  } else {
    if (d->xchg) {
      const Gathered X{recv, (long long)n, d->R, d->rank, d->m, 0};
      if (const int rc = ds_swap_launch(d, slot, iter, false, d->D.par, &X)) return rc;
    } else if (const int rc = ds_swap_launch(d, slot, iter, d->lslot_now, d->D.par, nullptr)) {
      return rc;
    }
    std::swap(d->D.idx, d->D.idx_out);  // the next iteration reads what the swaps wrote
    if (const int rc = ds_release(d, slot, sl.q)) return rc;
  }
  d->q_cons = sl.q + 1;  // the iteration's swap draws are on the stream, or deferred to the next ds_propose
  guard.armed = false;
  d->scv.notify_all();
  d->t_issue += now_s() - t0;
  if (d->P.log_on && iter > 10000 && iter % 100 == 0) {
    if (const int rc = ds_flush(d)) return rc;
    return ds_drain_events(d);
  }
  return 0;
}

extern "C" long hb_dsampler_step_begin(hb_dsampler* d, long iter, double* send, long cap) {
  if (!d) return hbx_set_error("hb_dsampler_step_begin: null");
  if (!d->xchg) return hbx_set_error("hb_dsampler_step_begin: sampler made by hb_dsampler_create, use hb_dsampler_step");
  return ds_begin(d, iter, send, cap);
}

extern "C" int hb_dsampler_step_end(hb_dsampler* d, long iter, const double* recv, long n) {
  if (!d) return hbx_set_error("hb_dsampler_step_end: null");
  return ds_end(d, iter, recv, n);
}

// one iteration, enqueued on the sampler's stream (no host wait)
extern "C" int hb_dsampler_step(hb_dsampler* d, long iter) {
  if (!d) return hbx_set_error("hb_dsampler_step: null");
  if (d->xchg) return hbx_set_error("hb_dsampler_step: sharded sampler, use step_begin / all-gather / step_end");
  const long rc = ds_begin(d, iter, nullptr, 0);
  if (rc < 0) {
    d->cur_iter = -1;
    return (int)rc;
  }
  return ds_end(d, iter, nullptr, 0);
}

// states / logL of the owned slots after the last step, the MAP tracker and
// the counters as :577-579 print them; synchronises
extern "C" int hb_dsampler_gather(hb_dsampler* d, double* x_slots, double* logl_slots, double* xmap,
                                  double* logLmap, long* stats4) {
  if (!d) return hbx_set_error("hb_dsampler_gather: null");
  if (const int rc = ds_flush(d)) return rc;
  const int nl = d->nl;
  hipStream_t s = d->st;
  DS_TRY(hipSetDevice(d->device), "hipSetDevice");
  ds_gather<<<(nl + kBlk - 1) / kBlk, kBlk, 0, s>>>(d->D, d->d_xs, d->d_ls, nullptr, nullptr);
  DS_TRY(hipGetLastError(), "gather");
  if (x_slots)
    DS_TRY(hipMemcpyAsync(x_slots, d->d_xs, sizeof(double) * nl * kNp, hipMemcpyDeviceToHost, s), "gather");
  if (logl_slots)
    DS_TRY(hipMemcpyAsync(logl_slots, d->d_ls, sizeof(double) * nl, hipMemcpyDeviceToHost, s), "gather");
  DS_TRY(hipMemcpyAsync(d->h_ctr, d->D.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s), "gather");
  DS_TRY(hipStreamSynchronize(s), "gather");
  if (xmap) memcpy(xmap, d->h_ctr->xmap, sizeof(double) * kNp);
  if (logLmap) *logLmap = d->h_ctr->logLmap;
  if (stats4)
    for (int i = 0; i < 4; ++i) stats4[i] = (long)d->h_ctr->snap[i];
  return 0;
}

#ifdef HB_DS_CLOCKS
extern "C" int hb_debug_dp_clocks(unsigned long long* out, int nslots) {
  if (nslots > 65536) nslots = 65536;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dp_clk), kDpClkWords * sizeof(unsigned long long) * nslots) == hipSuccess
             ? 0 : -1;
}
#endif
extern "C" int hb_dsampler_sync(hb_dsampler* d) {
  if (!d) return hbx_set_error("hb_dsampler_sync: null");
  if (const int rc = ds_flush(d)) return rc;
  DS_TRY(hipStreamSynchronize(d->st), "sync");
  return 0;
}

// internal (scripts/wall_probe.py): hbwall::apply_wall on n values, one wave
// per 64 of them, with each wave's shader cycles (cyc: ceil(n / 64) entries)
extern "C" int hbx_wall_probe(const double* v, const double* lo, const double* hi, long n, double* out,
                              long long* cyc) {
  if (n <= 0) return 0;
  const long nw = (n + 63) / 64;
  double *dv = nullptr, *dl = nullptr, *dh = nullptr, *dout = nullptr;
  long long* dc = nullptr;
  const size_t bytes = sizeof(double) * (size_t)n;
  hipError_t e = hipMalloc((void**)&dv, bytes);
  if (e == hipSuccess) e = hipMalloc((void**)&dl, bytes);
  if (e == hipSuccess) e = hipMalloc((void**)&dh, bytes);
  if (e == hipSuccess) e = hipMalloc((void**)&dout, bytes);
  if (e == hipSuccess) e = hipMalloc((void**)&dc, sizeof(long long) * (size_t)nw);
  if (e == hipSuccess) e = hipMemcpy(dv, v, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dl, lo, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dh, hi, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    ds_wall_probe<<<(unsigned)nw, 64>>>(dv, dl, dh, n, dout, dc);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(cyc, dc, sizeof(long long) * (size_t)nw, hipMemcpyDeviceToHost);
  for (void* p : {(void*)dv, (void*)dl, (void*)dh, (void*)dout, (void*)dc}) (void)hipFree(p);
  DS_TRY(e, "hbx_wall_probe");
  return 0;
}

// glibc-exact device math, for tests
extern "C" int hb_glibc_eval(int fn, const double* x, const double* y, long n, double* out) {
  if (n <= 0) return 0;
  double *dx = nullptr, *dy = nullptr, *dout = nullptr;
  const size_t bytes = sizeof(double) * (size_t)n;
  DS_TRY(hipMalloc((void**)&dx, bytes), "hipMalloc");
  DS_TRY(hipMalloc((void**)&dy, bytes), "hipMalloc");
  DS_TRY(hipMalloc((void**)&dout, bytes), "hipMalloc");
  hipError_t e = hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dy, y, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    ds_math_probe<<<(unsigned)((n + 255) / 256), 256>>>(fn, dx, dy, n, dout);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dout);
  DS_TRY(e, "hb_glibc_eval");
  return 0;
}

// ---------------------------------------------------------------------------
// hb_mcmc_run on the device: the mcmc_wrapper2.c loop with every iteration
// enqueued without a host round trip; the host joins every 100 iterations
// for the reference's file writes (:593-649) and progress lines (:575-589).
// ---------------------------------------------------------------------------
extern "C" int hb_mcmc_run_device(const hb_mcmc_cfg* cfg, hb_ctx* ctx, const double* t, const double* flux,
                                  long n, hb_mcmc_result* res) {
  if (!cfg || !ctx || cfg->nchains < 2 || cfg->npast < 2) return hbx_set_error("hb_mcmc_run_device: bad config");
  if (cfg->ladder == 0 && cfg->nchains > 2000) return hbx_set_error("hb_mcmc_run_device: ladder 0 needs W <= 2000");
  const int W = cfg->nchains;
  const long NITER = cfg->niter;
  hb_sampler* s = hb_sampler_create(cfg, 0, W);
  if (!s) return hbx_set_error("hb_mcmc_run_device: sampler");
  hb_writer* wr = nullptr;
  if (cfg->out_root && cfg->out_root[0]) {
    wr = hb_writer_open(cfg->out_root, cfg->run_id, cfg->run, W);
    if (!wr) {
      hb_sampler_destroy(s);
      return hbx_set_error("hb_mcmc_run_device: cannot open output files");
    }
    hb_sampler_attach_log(s, wr);
  }
  hb_dsampler* d = hb_dsampler_create(s, ctx);
  int rc = d ? 0 : -1;
  std::vector<double> xs((size_t)W * kNp), ls(W), model(n > 0 ? n : 1), xmap(kNp);
  double logLmap = 0;
  long st4[4];
  const double t_start = now_s();
  if (!rc) rc = hb_dsampler_init_logl(d);
  if (!rc && cfg->verbose) {
    rc = hb_dsampler_gather(d, nullptr, nullptr, xmap.data(), &logLmap, nullptr);
    if (!rc) printf("initial chi2 and likelihood %lf \t %lf\n", -2 * logLmap, logLmap);
  }
  for (long iter = 0; iter < NITER && !rc; ++iter) {
    rc = hb_dsampler_step(d, iter);
    if (rc) break;
    const bool show = cfg->verbose && iter % 1000 == 0;
    const bool write = wr && iter % 100 == 0;
    if (!(show || write)) continue;
    rc = hb_dsampler_gather(d, xs.data(), ls.data(), xmap.data(), &logLmap, st4);
    if (rc) break;
    if (show) {  // :575-589
      printf("%ld/%ld logL=%.10g acc=%.3g DEacc=%.3g", iter, NITER, ls[0], (double)st4[0] / ((double)st4[3]),
             (double)st4[1] / (double)st4[2]);
      printf("\n");
      printf("Parameter values: \n");
      for (int i = 0; i < 5; ++i) printf("%lf\t", xs[(size_t)(W > 10 ? 10 : W - 1) * kNp + i]);
      printf("\n");
    }
    if (write) {  // :593-649
      hb_writer_step(wr, iter, ls.data(), xs.data());
      if (n > 0 && t && flux) {
        rc = hb_light_curve_batch(ctx, xmap.data(), 1, model.data(), nullptr);
        if (rc) break;
        hb_writer_lc(wr, t, flux, model.data(), n);
      }
      hb_writer_pars(wr, 0, xs.data());
    }
  }
  if (!rc) rc = hb_dsampler_gather(d, xs.data(), ls.data(), xmap.data(), &logLmap, nullptr);
  if (!rc) rc = hb_dsampler_download(d);
  if (!rc && wr) {  // :655-681
    if (n > 0 && t && flux) {
      rc = hb_light_curve_batch(ctx, xmap.data(), 1, model.data(), nullptr);
      if (!rc) hb_writer_lc(wr, t, flux, model.data(), n);
    }
    hb_writer_pars(wr, 1, xs.data());
  }
  if (!rc && res) {
    long st6[6];
    hb_sampler_stats(s, st6);
    memcpy(res->xmap, xmap.data(), sizeof(double) * kNp);
    res->logLmap = logLmap;
    res->accepted = st6[4];
    res->swaps = st6[5];
    res->seconds_total = now_s() - t_start;
    res->seconds_loglik = -1.0;  // not separable: the likelihood runs inside the device loop
    res->loglik_evals = (long)W * (NITER + 1);
  }
  hb_dsampler_destroy(d);
  if (wr) hb_writer_close(wr);
  hb_sampler_destroy(s);
  return rc;
}
