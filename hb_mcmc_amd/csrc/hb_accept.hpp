// hb_accept.hpp -- the Hastings test and history write of mcmc_wrapper2.c
// (:492-546) for one slot, shared by the device sampler's ds_accept kernel
// (hb_dsampler.hip) and the likelihood kernel's fused epilogue
// (hb_eval_wave_kernel<..., ACC = true>, hb_kernels.hip), plus the sampler
// state types both need.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hb_glibc_math.hpp"

namespace hbds {

constexpr int kNp = 21;
constexpr int kEvCap = 1024;  // big-jump records between drains (<= 6 per iteration)

struct Counters {
  long long acc, DEacc, DEtrial, atrial, cold_acc, nswap;
  long long DEacc_tot, DEtrial_tot;  // sum over slots of DEacc_arr / DEtrial_arr
  long long acc_it;                  // cold-chain acceptances of this iteration
  long long snap[4];                 // {acc, DEacc, DEtrial, atrial} as printed at :577-579
  double logLmap;
  double xmap[kNp];
  int nev;
  int pad;
  // differential-evolution trials of chain 0 drawn by iteration q's proposals
  // (slot q & 1), folded into DEtrial_tot by q's bookkeeping (swap_tail): the
  // next iteration's proposals may run beside it (deferred swaps)
  long long de_trial_pend[2];
};

struct Event {  // LogSuspiciousJumps (:520-528) arguments
  long long iter;
  int chain, jtype, slot, pad;
  double H, alpha, tmp, lx, ly, px, py;
  double xo[kNp], xn[kNp];
};

// what the Hastings step of one iteration reads and writes (device pointers).
// A sampler may own only the slots [lo, lo + nl) of the W-slot ladder (one
// rank of a sharded run): arrays "by slot" hold those nl slots (local index
// j - lo), arrays "by chain" and idx/temp keep all W entries.
constexpr int kEvalOrdMax = 8192;  // walkers the eval launch takes by e (AccArgs::ecnt)
constexpr int kOrdBins = 64;       // one per lane (eval_slot_by_e)
// ints between two bins' counters: one 128-B line each (packed: measured 3.6 us slower per iteration)
constexpr int kEbinStride = 32;
// e bin of a proposal, descending e -> ascending bin (NaN -> last)
__device__ __forceinline__ int e_bin_desc(double e) {
  const double q = e * kOrdBins;
  const int b = q >= 0.0 ? (q < (double)kOrdBins ? (int)q : kOrdBins - 1) : 0;
  return kOrdBins - 1 - b;
}

// one tempering attempt of the level schedule: pair (b, b+1) and ln(beta) of
// its acceptance draw (beta itself is kept in a global-only array beside it)
struct SwapEnt {
  int b;
  int pad;
  double lnb;
};
// first slot of segment g of G over the owned slots [lo, lo + nl)
__host__ __device__ inline int seg_lo(int lo, int nl, int g, int G) { return lo + (int)((long long)nl * g / G); }
// segment holding slot x of [0, nl) (x clamped into the range)
__host__ __device__ inline int seg_of(int x, int nl, int G) {
  if (x < 0) x = 0;
  if (x > nl - 1) x = nl - 1;
  int g = (int)(((long long)x * G) / nl);
  while (g + 1 < G && seg_lo(0, nl, g + 1, G) <= x) ++g;
  while (g > 0 && seg_lo(0, nl, g, G) > x) --g;
  return g;
}

struct AccArgs {
  const int* idx;      // [W] slot -> chain
  double* logL;        // [W] by chain
  double* logP;        // [W] by chain
  const double* logPy; // [nl] by slot
  const double* temp;  // [W]
  const double* alpha2;
  const int* jump;
  const int* jtype;
  double* x;           // [W][21] by chain
  const double* y;     // [nl][21] by slot
  double* hist;        // [nl][NPAST][21] by slot
  int* DEacc_arr;
  Counters* ctr;
  Event* ev;
  int log_on, NPAST;
  long long iter;
  int lo;              // first owned slot
  int pad;
  // eval wave -> local slot by descending e (null: wave w takes slot w):
  // ds_propose files slot j under bin b = e_bin_desc(e_j) at
  // elist[b * ecap + ecnt[b]++].  The counters alternate between two buffers
  // by iteration; this launch clears the next iteration's (ecnt_next, read by
  // the previous launch, filed by the next ds_propose)
  const int* ecnt;     // [kOrdBins]
  const int* elist;    // [kOrdBins][ecap]
  int ecap, pad2;
  double* Lslot;       // [W] logL of the chain in slot j after its Hastings test (null: not kept)
  int* ecnt_next;      // [kOrdBins] (null: none)
};

// Eval wave s of the device sampler takes the s-th slot of the bins in order
// (descending e).  The launch is one resident round of waves, four per SIMD,
// so it lasts as long as the SIMD whose walkers cost most; cost follows e
// (high e leaves the warm Kepler chains for the cold path), and waves taking
// the walkers by descending e give every SIMD walkers from the whole e range
// (sampler states of a 200-iteration run: 53 us in slot order, 47 us sorted;
// bins by expected cost from the records instead -- cold path by e, warm
// chains, Roche walkers last -- measured the same: 0.0918-0.0923 ms per
// iteration either way, profiles/r05/r05d_ds_cost_order_ab.txt).
// The order within a bin is immaterial: a wave's result depends on its
// walker only.  One load and a wave scan over the 64 bin counts.
__device__ __forceinline__ int eval_slot_by_e(const AccArgs& A, int s, int lane) {
  const int c = A.ecnt[lane * kEbinStride];
  int incl = c;
#pragma unroll
  for (int d = 1; d < kOrdBins; d <<= 1) {
    const int o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  const unsigned long long m = __ballot(incl > s);
  if (m == 0ull) return s;  // not reached: the bins hold every slot
  const int b = __builtin_ctzll(m);
  const int start = __shfl(incl - c, b);
  return __builtin_amdgcn_readfirstlane(A.elist[(size_t)b * A.ecap + (s - start)]);
}

// Everything the Hastings test of local slot j reads besides the new logL.
// None of it depends on the likelihood, so the eval kernel loads it when the
// wave starts and the test at the end of the wave waits on nothing but exp.
struct AccPre {
  int jg, chain;
  double lx, temp, dlp, alpha, xo, yn;
};
// the wave-uniform operands only (the per-lane rows: accept_prefetch_rows)
__device__ inline AccPre accept_prefetch_uniform(const AccArgs& A, int j) {
  AccPre p;
  p.jg = j + A.lo;
  p.chain = A.idx[p.jg];
  p.lx = A.logL[p.chain];
  p.temp = A.temp[p.jg];
  p.dlp = A.logPy[j] - A.logP[p.chain];
  p.alpha = A.alpha2[j];
  p.xo = 0.0;
  p.yn = 0.0;
  return p;
}
__device__ inline void accept_prefetch_rows(const AccArgs& A, int j, int lane, AccPre& p) {
  if (lane < kNp) {
    p.xo = A.x[(size_t)p.chain * kNp + lane];
    p.yn = A.y[(size_t)j * kNp + lane];
  }
}
__device__ inline AccPre accept_prefetch(const AccArgs& A, int j, int lane) {
  AccPre p = accept_prefetch_uniform(A, j);
  accept_prefetch_rows(A, j, lane, p);
  return p;
}

// Hastings test of local slot j (global slot lo + j) whose proposal has logL
// ly, by one wave: lane n < 21 moves coordinate n (x[chain] = y if accepted,
// history row k = x[chain]); lane 0 does the scalar bookkeeping.  Same
// operations and order of effects as ds_accept.
// returns whether the proposal was accepted
__device__ inline bool accept_slot_wave_pre(const AccArgs& A, int j, double ly, int lane, const AccPre& p) {
  const int jg = p.jg;
  const int chain = p.chain;
  const double lx = p.lx;
  const double H = hbglibc::exp((ly - lx) / p.temp + p.dlp);
  const bool acc = p.alpha <= H;
  const int k = (int)(A.iter - (A.iter / A.NPAST) * A.NPAST);
  const double xo = p.xo, yn = p.yn;
  if (acc) {
    if ((lx / ly <= 0.5) && (A.iter > 10000) && (jg <= 5) && A.log_on) {
      int e = 0;
      if (lane == 0) e = atomicAdd(&A.ctr->nev, 1);
      e = __shfl(e, 0);
      if (e < kEvCap) {
        Event& ev = A.ev[e];
        if (lane == 0) {
          ev.iter = A.iter;
          ev.chain = chain;
          ev.jtype = A.jtype[j];
          ev.slot = jg;
          ev.H = H;
          ev.alpha = A.alpha2[j];
          ev.tmp = A.temp[jg];
          ev.lx = lx;
          ev.ly = ly;
          ev.px = A.logP[chain];
          ev.py = A.logPy[j];
        }
        if (lane < kNp) {
          ev.xo[lane] = xo;
          ev.xn[lane] = yn;
        }
      }
    }
    if (lane == 0) {
      if (chain == 0) atomicAdd((unsigned long long*)&A.ctr->acc_it, 1ull);
      A.logL[chain] = ly;
      A.logP[chain] = A.logPy[j];
      if ((A.jump[j] == 1) && (chain == 0)) {
        A.DEacc_arr[j]++;
        atomicAdd((unsigned long long*)&A.ctr->DEacc_tot, 1ull);
      }
    }
  }
  if (lane < kNp) {
    const double v = acc ? yn : xo;
    if (acc) A.x[(size_t)chain * kNp + lane] = v;
    A.hist[((size_t)j * A.NPAST + k) * kNp + lane] = v;
  }
  // logL by slot for the swap step (ds_swap_seg stages it without the
  // dependent index[] -> logL[chain] load)
  if (lane == 0 && A.Lslot != nullptr) A.Lslot[jg] = acc ? ly : lx;
  return acc;
}
__device__ inline void accept_slot_wave(const AccArgs& A, int j, double ly, int lane) {
  accept_slot_wave_pre(A, j, ly, lane, accept_prefetch(A, j, lane));
}

}  // namespace hbds
