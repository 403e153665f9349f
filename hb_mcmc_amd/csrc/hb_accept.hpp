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
#ifndef HB_EBIN_STRIDE
#define HB_EBIN_STRIDE 32  // ints between two bins' counters: one 128-B line each (1: packed, measured 3.6 us slower per iteration)
#endif
constexpr int kEbinStride = HB_EBIN_STRIDE;
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
  // elist[b * ecap + ecnt[b]++]; ds_swap clears ecnt for the next iteration
  const int* ecnt;     // [kOrdBins]
  const int* elist;    // [kOrdBins][ecap]
  int ecap, pad2;
  // Tempering swaps at the launch's tail (one-process samplers; tcnt null:
  // the caller launches ds_swap_seg).  The iteration's level schedule as
  // ds_swap_seg reads it, the pair factors, and what the swap step writes.
  int* tcnt;           // [G + 2] cone counters of the segments, segments done (zero between launches), chain in slot 0
  double* Lslot;       // [W + 1] logL of the chain in slot j after its Hastings test (null: not kept); [W]: the swap tail's logL of slot 0 after the swaps
  const int* soff;     // [G nlv + 1]
  const SwapEnt* ent;
  const double* betas;
  const double* hs;    // [W] (T_b - T_b+1) / (T_b T_b+1)
  int* idx_out;        // [W] next iteration's index[]
  int* DEtrial_arr;    // [nl]
  int* ecnt_w;         // = ecnt, cleared by the last segment
  int W, nlv, G, nl;
};

// Eval wave s of the device sampler takes the s-th slot of the bins in order
// (descending e).  The launch is one resident round of waves, four per SIMD,
// so it lasts as long as the SIMD whose walkers cost most; cost follows e
// (high e leaves the warm Kepler chains for the cold path), and waves taking
// the walkers by descending e give every SIMD walkers from the whole e range
// (sampler states of a 200-iteration run: 53 us in slot order, 47 us sorted).
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
        if (A.tcnt) atomicAdd(&A.DEacc_arr[j], 1);  // the swap tail may reset it in this launch
        else A.DEacc_arr[j]++;
        atomicAdd((unsigned long long*)&A.ctr->DEacc_tot, 1ull);
      }
    }
  }
  if (lane < kNp) {
    const double v = acc ? yn : xo;
    if (acc) {
      if (A.tcnt) __hip_atomic_store(&A.x[(size_t)chain * kNp + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else A.x[(size_t)chain * kNp + lane] = v;  // (the swap tail's MAP tracker reads it device-coherently)
    }
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

// ---------------------------------------------------------------------------
// Tempering swaps (ptmcmc, mcmc_wrapper2.c:768-817) at the tail of the
// likelihood launch, for a one-process sampler (lo = 0, nl = W).  Segment g
// of the level schedule (ds_swap_seg in hb_dsampler.hip: the cone argument,
// the LDS layout and the per-attempt test are the same) can be replayed as
// soon as every slot of its cone [sl - nlv, sh + nlv) has had its Hastings
// test.  So after its test each eval wave counts its slot in the (at most a
// few) cones holding it; the wave whose count completes a cone replays that
// segment in its own LDS (the model slab is dead by then), one wave wide.
// The wave completing the last segment does the iteration's bookkeeping and
// zeroes the counters for the next launch.
//
// Coherence across the eight XCDs' L2s without write-back fences (an
// agent-scope release fence is an L2 write-back per wave: measured 0.143 vs
// 0.095 ms per iteration): every value one wave hands to another inside the
// launch goes through device-scope atomic stores/loads (sc1: written through
// / read past the non-coherent L2), and a wave waits for its own stores to be
// acknowledged (s_waitcnt vmcnt(0)) before the counter atomics that publish
// them.  The values: the post-test logL by slot (Lslot), the chain state x of
// an accepted proposal (for the MAP tracker), DEacc_arr, the chain in slot 0
// and its logL after the swaps, and the counters.
// ---------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ void dst(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class T>
__device__ __forceinline__ T dld(const T* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void wait_stores() { __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__host__ __device__ inline size_t tail_lds_bytes(size_t maxent, size_t wc_max) {
  return sizeof(SwapEnt) * maxent + (2 * sizeof(double) + sizeof(int)) * wc_max;
}

__device__ inline void tail_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline void tail_replay(const AccArgs& A, int g, int lane, unsigned char* lds) {
  const int W = A.W, nlv = A.nlv, G = A.G;
  const int sl = seg_lo(0, A.nl, g, G), sh = seg_lo(0, A.nl, g + 1, G);
  const int clo = max(0, sl - nlv), chi = min(W, sh + nlv), Wc = chi - clo;
  const int eb = A.soff[g * nlv], ne = A.soff[g * nlv + nlv] - eb;
  SwapEnt* sE = reinterpret_cast<SwapEnt*>(lds);
  double* cL = reinterpret_cast<double*>(lds + sizeof(SwapEnt) * (size_t)ne);
  double* cH = cL + Wc;
  int* cC = reinterpret_cast<int*>(cH + Wc);
  for (int q = lane; q < ne; q += 64) sE[q] = A.ent[eb + q];
  for (int i = lane; i < Wc; i += 64) {
    cC[i] = A.idx[clo + i];
    cH[i] = A.hs[clo + i];
    cL[i] = dld(&A.Lslot[clo + i]);
  }
  tail_lds_sync();
  int nacc = 0;
  for (int lv = 0; lv < nlv; ++lv) {
    const int e0 = A.soff[g * nlv + lv] - eb, e1 = A.soff[g * nlv + lv + 1] - eb;
    for (int q = e0 + lane; q < e1; q += 64) {  // the attempts of a level touch disjoint pairs
      const int b = sE[q].b;
      const double lnb = sE[q].lnb;
      const int bl = b - clo, al = bl + 1;
      const double lb = cL[bl], la = cL[al];
      const double x = (lb - la) * cH[bl];  // :803
      bool acc;
      const double dl = 1e-12 * (1.0 + fabs(lnb));
      if (lnb > -HUGE_VAL && x >= lnb + dl) acc = true;
      else if (lnb > -HUGE_VAL && x <= lnb - dl) acc = false;
      else acc = hbglibc::exp(x) >= A.betas[eb + q];
      if (acc) {
        const int ca = cC[al], cb = cC[bl];
        cL[al] = lb;
        cL[bl] = la;
        cC[al] = cb;
        cC[bl] = ca;
        if (b >= sl && b < sh) ++nacc;
      }
    }
    tail_lds_sync();
  }
  for (int s = sl + lane; s < sh; s += 64) A.idx_out[s] = cC[s - clo];
  if (A.iter % 100 == 0)
    for (int s = sl + lane; s < sh; s += 64) {
      dst(&A.DEacc_arr[s], 0);
      A.DEtrial_arr[s] = 0;
    }
  if (sl == 0 && lane == 0) {  // the chain now in slot 0 and its logL, for the bookkeeping
    dst(&A.tcnt[G + 1], cC[0 - clo]);
    dst(&A.Lslot[W], cL[0 - clo]);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) nacc += __shfl_xor(nacc, off, 64);
  if (lane == 0 && nacc) atomicAdd((unsigned long long*)&A.ctr->nswap, (unsigned long long)nacc);
}

// the per-iteration bookkeeping after the swaps (:551-572, :590, :622-629),
// as ds_swap_seg's swap_tail, by the wave completing the last segment
__device__ inline void tail_bookkeeping(const AccArgs& A, int lane) {
  if (A.ecnt_w != nullptr && lane < kOrdBins) A.ecnt_w[lane * kEbinStride] = 0;  // every eval wave has read them
  Counters* C = A.ctr;
  const int c0 = dld(&A.tcnt[A.G + 1]);
  const double L0 = dld(&A.Lslot[A.W]);
  double xc = 0.0;
  if (lane < kNp) xc = dld(&A.x[(size_t)c0 * kNp + lane]);
  const bool map = L0 > C->logLmap;  // :565-572
  if (map && lane < kNp) C->xmap[lane] = xc;
  for (int g = lane; g <= A.G + 1; g += 64) dst(&A.tcnt[g], 0);  // for the next launch
  if (lane != 0) return;
  const long long acc_it = dld(&C->acc_it), de_tot = dld(&C->DEacc_tot), dt_tot = dld(&C->DEtrial_tot);
  C->acc += acc_it;
  C->cold_acc += acc_it;
  C->DEacc += de_tot;
  C->DEtrial += dt_tot;
  dst(&C->acc_it, 0ll);
  C->snap[0] = C->acc;
  C->snap[1] = C->DEacc;
  C->snap[2] = C->DEtrial;
  C->snap[3] = C->atrial;
  if (map) C->logLmap = L0;
  C->atrial++;
  if (A.iter % 100 == 0) {
    C->acc = C->atrial = 0;
    dst(&C->DEacc_tot, 0ll);
    dst(&C->DEtrial_tot, 0ll);
  }
}

// after the Hastings test of local slot j (logL of its chain now lnew):
// publish lnew, count j in its cones, replay the segments this wave
// completes, and the bookkeeping if it completes the last
#ifndef HB_SWAP_TAIL
#define HB_SWAP_TAIL 0  // 1: compile the swap tail into the fused eval kernel (experiment, measured slower)
#endif
#ifndef HB_TAIL_NOINLINE
#define HB_TAIL_NOINLINE 0  // 1: the swap tail as an out-of-line call (measured slower)
#endif
#if HB_TAIL_NOINLINE
__device__ __attribute__((noinline))
#else
__device__ inline
#endif
void swap_tail_wave(const AccArgs& A, int j, double lnew, int lane, unsigned char* lds) {
  const int nlv = A.nlv, G = A.G;
  if (lane == 0) dst(&A.Lslot[j], lnew);
  wait_stores();  // this wave's device-scope stores are acknowledged before its counts
  const int g0 = seg_of(j - nlv, A.nl, G), g1 = seg_of(j + nlv, A.nl, G);
  bool done = false;
  const int g = g0 + lane;
  if (g <= g1) {
    const int sl = seg_lo(0, A.nl, g, G), sh = seg_lo(0, A.nl, g + 1, G);
    const int wc = min(A.W, sh + nlv) - max(0, sl - nlv);
    if (sl - nlv <= j && j < sh + nlv) done = atomicAdd(&A.tcnt[g], 1) + 1 == wc;
  }
  unsigned long long m = __ballot(done);
  if (m == 0ull) return;
  int fin = 0;
  while (m) {
    const int k = __builtin_ctzll(m);
    m &= m - 1ull;
    tail_replay(A, g0 + k, lane, lds);
    tail_lds_sync();  // the next segment restages the same LDS
    wait_stores();
    int last = 0;
    if (lane == 0) last = atomicAdd(&A.tcnt[G], 1) + 1 == G;
    fin |= __shfl(last, 0);
  }
  if (fin) tail_bookkeeping(A, lane);
}

}  // namespace hbds
