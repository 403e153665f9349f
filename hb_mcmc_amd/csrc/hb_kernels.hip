// hb_kernels.hip -- gfx950 kernels for the HB light-curve log-likelihood.
//
//   hb_prep_kernel      WalkerConst (hb_device.hpp) by prep groups (hb_prep.hpp)
//   hb_eval_kernel<NW>  one workgroup of NW waves per walker:
//                         1. model flux for every cadence (t streamed from
//                            HBM/L2, coalesced), kept in LDS (or an HBM slab
//                            when N*8 B exceeds the LDS budget);
//                         2. exact median by radix-select on order-preserving
//                            64-bit keys, 8-bit digits starting below the
//                            common prefix of min/max, LDS histogram
//                            (replaces quickSort, likelihood3.c:86-105);
//                         3. normalise + blend (:679-685) and chi^2 with a
//                            wave-shuffle + LDS reduction (:822-832), then the
//                            Gaia term and Roche override (:834-869).
//
// All launches are asynchronous on the caller's stream and allocation-free
// once hb_reserve() sized the workspace.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "hb_accept.hpp"
#include "hb_device.hpp"
#include "hb_internal.hpp"
#ifdef HB_WAVE_CLOCKS
// the fused launch's prologue, 16 marks per workgroup (see HB_PCLK below);
// prep-role marks 5..8 (phase 1 done, role 0..3), 9..12 (phase 2), 13 (wave
// 0: records combined)
__device__ unsigned long long hb_pro_clk[16 * 4096];
#define HB_PREP_MARK(i)                                                                      \
  do {                                                                                       \
    if ((i) != 13 || (threadIdx.x >> 6) == 0)                                                \
      if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                      \
        hb_pro_clk[16 * blockIdx.x + (i)] = __builtin_amdgcn_s_memtime();                    \
  } while (0)
#endif
#include "hb_prep.hpp"

using namespace hbdev;

#ifndef HB_K
#define HB_K 4  // cadences interleaved per lane in the model loop (4: +1% over 2 on MI355X, 117 VGPRs)
#endif
#ifndef HB_WAVES_PER_EU
#define HB_WAVES_PER_EU 4  // keep the wave kernel at <= 128 VGPRs: 4 waves per SIMD
#endif
#if HB_WAVES_PER_EU > 0
#define HB_WPE_ATTR __attribute__((amdgpu_waves_per_eu(HB_WAVES_PER_EU)))
#else
#define HB_WPE_ATTR
#endif
#ifndef HB_UNCOND_PH
#define HB_UNCOND_PH 0  // 1: unpredicated table loads (measured slower: register pressure)
#endif
#ifndef HB_FULLTILE
#define HB_FULLTILE 1  // full K*64 tiles store without per-cadence bounds tests
#endif
#ifndef HB_ABLATE_MODEL
#define HB_ABLATE_MODEL 0
#endif
#ifndef HB_ABLATE_SELECT
#define HB_ABLATE_SELECT 0
#endif
#ifndef HB_ACC_PRE
#define HB_ACC_PRE 1  // fused Hastings test: operands loaded at wave start (see hb_eval_wave_kernel)
#endif
#ifndef HB_PRIO
#define HB_PRIO 1  // wave pacing (Pacer): 0 off, 1 by own quartile, 2 by lead over the SIMD's slowest wave
#endif
// LDS ordering among the lanes of ONE wave (the one-wave-per-walker kernel may
// share its workgroup with other walkers' waves, which must not be waited for)
#define HB_WSYNC()                                        \
  do {                                                    \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
    __builtin_amdgcn_wave_barrier();                      \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
  } while (0)
// Experiment builds only (HB_WAVE_CLOCKS): per-wave shader clock at entry and
// exit plus HW_ID / XCC_ID, read back by hb_debug_wave_clocks().
#ifdef HB_WAVE_CLOCKS
// 8 words per wave: start, phase marks 0..2 (after the model pass, the keys,
// the select; 0 if not reached), end, HW_ID, XCC_ID, mark 3 (the model loop's
// end, before the deferred queue is applied)
__device__ unsigned long long hb_wave_clk[8 * 65536];
#define HB_CLK_BEGIN()                                     \
  const unsigned long long clk0_ = __builtin_amdgcn_s_memtime(); \
  unsigned long long clkm_[4] = {0ull, 0ull, 0ull, 0ull}
#define HB_CLK_MARK(i) clkm_[(i)] = __builtin_amdgcn_s_memtime()
#define HB_CLK_END(wv)                                                                  \
  do {                                                                                  \
    const unsigned long long clk1_ = __builtin_amdgcn_s_memtime();                      \
    if ((threadIdx.x & 63) == 0 && (wv) < 65536) {                                      \
      hb_wave_clk[8 * (wv) + 0] = clk0_;                                                \
      hb_wave_clk[8 * (wv) + 1] = clkm_[0];                                             \
      hb_wave_clk[8 * (wv) + 2] = clkm_[1];                                             \
      hb_wave_clk[8 * (wv) + 3] = clkm_[2];                                             \
      hb_wave_clk[8 * (wv) + 4] = clk1_;                                                \
      hb_wave_clk[8 * (wv) + 5] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);  \
      hb_wave_clk[8 * (wv) + 6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20); \
      hb_wave_clk[8 * (wv) + 7] = clkm_[3];                                             \
    }                                                                                   \
  } while (0)
// the fused launch's prologue (wave 0 of each workgroup): 0 entry, 1 parameters
// in LDS, 2 records in LDS (prep_records done), 3 after the last barrier,
// 4 the table waves' work done (thread 256); 5.. the prep roles (HB_PREP_MARK)
#define HB_PCLK(i, thr)                                                                \
  do {                                                                                 \
    if (threadIdx.x == (thr) && blockIdx.x < 4096)                                     \
      hb_pro_clk[16 * blockIdx.x + (i)] = __builtin_amdgcn_s_memtime();                \
  } while (0)
#else
#define HB_PCLK(i, thr) do { } while (0)
#define HB_CLK_BEGIN() do { } while (0)
#define HB_CLK_MARK(i) do { } while (0)
#define HB_CLK_END(wv) do { } while (0)
#endif

// whether this build of the eval kernel carries the swap tail (hb_accept.hpp)
extern "C" int hbx_swap_tail_compiled(void) { return HB_SWAP_TAIL; }

namespace hbk {

// ---------------------------------------------------------------------------
// kernel 1: per-walker constants (hb_prep.hpp), kPrepWalkers walkers per
// 256-thread workgroup (a prep group: four role waves, lane = walker), so
// W = 4096 launches 256 workgroups, one per CU.  Parameters and records move
// through LDS so the HBM accesses coalesce.  The device sampler computes the
// same records in ds_propose's epilogue instead (no launch per iteration).
// ---------------------------------------------------------------------------
#ifndef HB_PREP_W
#define HB_PREP_W 16
#endif
constexpr int kPrepWalkers = HB_PREP_W;  // walkers per prep workgroup (small batches)
constexpr int kPrepThreads = 64 * kPrepRoles;

// NW walkers per workgroup: kPrepWalkers, or 32 / 64 for batches that still
// fill 256 workgroups with them (C4, C5: one round instead of two or four)
// LIST (catalog, one size class): the launch's walkers are list[0..nwalk),
// their magnitude data gathered into LDS; a walker's table period is its
// target's first walker's (the catalog's evals evaluate the table entries in
// place, so no table is written)
template <int NW, bool LIST = false>
__global__ __launch_bounds__(kPrepThreads) void hb_prep_kernel(const double* __restrict__ params,
                                                              int nwalk, MagArgs ma,
                                                              WalkerConst* __restrict__ out,
                                                              const TargetDesc* __restrict__ tab,
                                                              const int* __restrict__ wt,
                                                              const double* __restrict__ tcad, int ncad,
                                                              double2* __restrict__ ph,
                                                              const int* __restrict__ w0, int ntargets,
                                                              double* __restrict__ tab_pc_out,
                                                              const int* __restrict__ list) {
  constexpr int kPrepWalkers = NW;
  __shared__ PrepShared<kPrepWalkers> L;
  __shared__ double mg_s[LIST ? 3 * NW : 1];
  __shared__ int wl_s[LIST ? NW : 1], wtl_s[LIST ? NW : 1];
  const int G = (int)gridDim.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int base = blockIdx.x * kPrepWalkers;
  const int nb = min(kPrepWalkers, nwalk - base);
  if constexpr (LIST) {
    if (tid < NW) {
      const int wk = tid < nb ? list[base + tid] : 0;
      const int tg = wt[wk];
      wl_s[tid] = wk;
      wtl_s[tid] = tg;
      mg_s[tid] = tab[tg].dist;
      mg_s[NW + tid] = tab[tg].gmag;
      mg_s[2 * NW + tid] = tab[tg].gerr;
    }
    __syncthreads();
  }
  // wave 2 writes a single context's shared-period phase table in its slack;
  // its first operands are in flight with the parameters
  const bool tabwave = ph != nullptr && tab == nullptr && (tid >> 6) == 2;
  double t_first = 0.0, lp0 = 0.0;
  if (tabwave) {
    const int i0 = blockIdx.x + G * lane;
    if (i0 < ncad) t_first = tcad[i0];
    lp0 = params[2];
  }
  {  // all loads in flight before the first LDS write (a rolled loop serialises on vmcnt(0))
    constexpr int U = (kPrepWalkers * kNpars + kPrepThreads - 1) / kPrepThreads;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kPrepThreads;
      if constexpr (LIST) {
        const int j = i / kNpars;
        v[u] = i < nb * kNpars ? params[(size_t)wl_s[j] * kNpars + (i - j * kNpars)] : 0.0;
      } else {
        v[u] = i < nb * kNpars ? params[(size_t)base * kNpars + i] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kPrepThreads;
      if (i < nb * kNpars) L.sp[i] = v[u];
    }
  }
  __syncthreads();
  // the table period: walker 0's (single context) or the first walker's of
  // the walker's target in this batch (catalog)
  auto tab_pc = [&](int j) -> double {
    if constexpr (LIST) return exp10(params[(size_t)w0[wtl_s[j]] * kNpars + 2]) * kDay;
    if (ph == nullptr) return __builtin_nan("");
    return exp10(params[(tab ? (size_t)w0[wt[base + j]] * kNpars : 0) + 2]) * kDay;
  };
  // ph[i] = (sin, cos)(t_i DAY 2pi/Pc0) for the period of walker 0, entries
  // dealt round-robin over the workgroups' wave-2 lanes
  auto slack = [&]() {
    if (!tabwave) return;
    const double Pc0 = exp10(lp0) * kDay;
    const double mA0 = kTwoPi / Pc0;
    if (blockIdx.x == 0 && lane == 0 && tab_pc_out != nullptr) *tab_pc_out = Pc0;
    double ti = t_first;
    for (int i = blockIdx.x + G * lane; i < ncad; i += G * 64) {
      double sv, cv;
      sincos_table((ti * kDay) * mA0, sv, cv);
      ph[i] = make_double2(sv, cv);
      if (i + G * 64 < ncad) ti = tcad[i + G * 64];
    }
  };
  if constexpr (LIST)
    prep_records<kPrepWalkers>(L, nb, ma, nullptr, nullptr, 0, tab_pc, slack, PrepNoIdle(), mg_s);
  else
    prep_records<kPrepWalkers>(L, nb, ma, tab, wt, base, tab_pc, slack);
  {
    double* dst = reinterpret_cast<double*>(out) + (size_t)base * kWcDoubles;
    constexpr int U = (kPrepWalkers * kWcDoubles + kPrepThreads - 1) / kPrepThreads;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kPrepThreads;
      const int jw = i / kWcDoubles;  // record rows of kSoStride doubles in LDS
      v[u] = i < nb * kWcDoubles ? L.so[jw * kSoStride + (i - jw * kWcDoubles)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kPrepThreads;
      if (i < nb * kWcDoubles) {
        if constexpr (LIST) {
          const int j = i / kWcDoubles;
          reinterpret_cast<double*>(out)[(size_t)wl_s[j] * kWcDoubles + (i - j * kWcDoubles)] = v[u];
        } else {
          dst[i] = v[u];
        }
      }
    }
  }
  if constexpr (LIST) return;
  // Catalog phase table (WalkerConst::tab), written after the walker records
  // so its latency overlaps their stores: per target k, for the period of its
  // first walker w0[k] in this batch (-1: no walkers), ph[i] = (sin, cos)(t_i
  // DAY 2pi/Pc0) over its slice of the concatenated arrays.  (A single
  // context's table is written by wave 2 above.)
  if (ph && tab != nullptr) {
    for (int k = blockIdx.x; k < ntargets; k += G) {
      if (w0[k] < 0) continue;
      const double mA0 = kTwoPi / (exp10(params[(size_t)w0[k] * kNpars + 2]) * kDay);
      const long off = tab[k].off;
      for (int i = tid; i < (int)tab[k].n; i += blockDim.x) {
        double sv, cv;
        sincos_table((tcad[off + i] * kDay) * mA0, sv, cv);
        ph[off + i] = make_double2(sv, cv);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// block-level helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    uint64_t o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    uint64_t o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Model flux for cadences tid, tid+NT, ... : HB_K interleaved cadences per lane
// per iteration (ILP for the fp64 Kepler chains), next iteration's times
// prefetched; values go to vals[], min/max order keys returned per lane.
template <int NT>
__device__ __forceinline__ void model_pass(const double* __restrict__ t, const double2* __restrict__ ph, int n,
                                           const WalkerConst& w, double* vals, int tid, uint64_t& kmn_out,
                                           uint64_t& kmx_out) {
  constexpr int K = HB_K;
  const bool tab = (ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  // running min/max as doubles (v_min/v_max_f64); NaN lanes are tracked and
  // the order keys recomputed from vals[] in that (never observed) case
  double vmn = __builtin_inf(), vmx = -__builtin_inf();
  bool nan = false;
  const int last = n - 1;
  // table entries load unconditionally: off the table, from t[0..1] (ignored)
#if HB_UNCOND_PH
  const double2* __restrict__ php = tab ? ph : reinterpret_cast<const double2*>(t);
  const int pmask = tab ? ~0 : 0;
#define HB_PH_LOAD(i) php[(i) & pmask]
#else
#define HB_PH_LOAD(i) (tab ? ph[i] : make_double2(0.0, 1.0))
#endif
  double tk[K];
  double2 pk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = min(k * NT + tid, last);
    tk[k] = t[i];
    pk[k] = HB_PH_LOAD(i);
  }
  for (int base = 0; base < n; base += K * NT) {
    double tn[K];
    double2 pn[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = min(base + (K + k) * NT + tid, last);
      tn[k] = t[i];
      pn[k] = HB_PH_LOAD(i);
    }
    double v[K];
    bool bad;
#if HB_ABLATE_MODEL  // experiment builds only: trivial model, same data flow
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = tk[k] * w.kb + w.kr0;
    bad = false;
#else
#if HB_SPLIT_LIVE
    __asm__ volatile("" ::: "memory");  // walker constants reloaded per tile (see hb_cadence_flux_k)
#endif
    hb_cadence_flux_k<K>(tk, pk, tab, w, v, bad);
#endif
    if (wave_any(bad)) {  // out-of-domain angles: reference-order ocml path
      if (bad) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = hb_cadence_flux_slow(tk[k], &w);
      }
    }
    if (HB_FULLTILE && base + K * NT <= n) {  // full tile: no per-cadence bounds test
#pragma unroll
      for (int k = 0; k < K; ++k) {
        vals[base + k * NT + tid] = v[k];
        vmn = fmin(vmn, v[k]);
        vmx = fmax(vmx, v[k]);
        nan |= v[k] != v[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int i = base + k * NT + tid;
        if (i < n) {
          vals[i] = v[k];
          vmn = fmin(vmn, v[k]);
          vmx = fmax(vmx, v[k]);
          nan |= v[k] != v[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      tk[k] = tn[k];
      pk[k] = pn[k];
    }
  }
  // keys of the extremes; -0.0 / +0.0 compare equal but key apart: take the
  // outer key of a zero extreme so [kmn, kmx] brackets every key
  uint64_t kmn = dkey(vmn == 0.0 ? -0.0 : vmn), kmx = dkey(vmx == 0.0 ? 0.0 : vmx);
  if (wave_any(nan)) {
    kmn = ~0ull;
    kmx = 0ull;
    for (int i = tid; i < n; i += NT) {
      const uint64_t key = dkey(vals[i]);
      kmn = key < kmn ? key : kmn;
      kmx = key > kmx ? key : kmx;
    }
  }
  kmn_out = kmn;
  kmx_out = kmx;
}

// One-wave kernel: lane l owns the rc = ceil(n/64) consecutive cadences
// l*rc .. l*rc + rc - 1 (its row of the LDS slab, later its select keys).
// The chain path solves a row as KC chains whose Kepler starts are warm
// (hb_cadence_flux_chain) after each chain's first cadence.  Row stride
// rc | 1: an odd stride spreads a wave's accesses at one row position over
// the banks, and position c of a lane's row sits at a constant offset from
// the row's start, so the key loads take immediate offsets (no per-key
// address arithmetic).  The slab is ~n * 8 bytes, so short light curves of a
// catalog class keep more waves per CU.
#ifndef HB_KC
#define HB_KC 2  // chains per lane
#endif
#ifndef HB_PAIR_KC
#define HB_PAIR_KC HB_KC  // experiment knob: Kepler chains per lane in the pair kernel
#endif
#ifndef HB_ODD_STRIDE
#define HB_ODD_STRIDE 1  // 0: power-of-two rows stored at c ^ (lane mod rc) (stride rc)
#endif
struct Rows {
  int rc;      // cadences per lane row
  int stride;  // row stride [doubles]
  int swz;     // XOR swizzle mask (HB_ODD_STRIDE == 0, power-of-two rc: rc - 1; else 0)
  float rcp;   // 1 / rc (row of cadence i, i < 2^11: exact after rounding)
  int live;    // rows holding cadences: ceil(n / rc) (the rows kernel stores no others)
};
constexpr long kRowsLdsCap = 163840 - 2048;  // the rows kernel's slab, below its candidates and shared words
__host__ __device__ __forceinline__ int rows_stride(int rc) {
  return (HB_ODD_STRIDE || (rc & (rc - 1)) != 0) ? (rc | 1) : rc;
}
// nr lane rows per walker: 64 (one wave) or 128 (a pair of waves, WPW = 2)
__device__ __forceinline__ Rows make_rows(int n, int nr = 64) {
  Rows r;
  r.rc = (n + nr - 1) / nr;
  r.stride = rows_stride(r.rc);
  r.live = (n + r.rc - 1) / r.rc;
  // many rows (the rows kernel, nr > 128): the odd pad only while the live rows fit the LDS
  if (nr > 128 && (long)r.live * r.stride * 8 > kRowsLdsCap) r.stride = r.rc;
  r.swz = (!HB_ODD_STRIDE && (r.rc & (r.rc - 1)) == 0) ? r.rc - 1 : 0;
  r.rcp = 1.0f / (float)r.rc;
  return r;
}
__device__ __forceinline__ int slab_pos(const Rows& r, int lane, int c) {
  return HB_ODD_STRIDE ? lane * r.stride + c : lane * r.stride + (c ^ (lane & r.swz));
}
// slab position of cadence i: row q = i / rc by the fp32 reciprocal
// ((i + 0.5) / rc is >= 1/(2 rc) away from an integer, far above its error)
__device__ __forceinline__ int slab_pos_of(const Rows& r, int i) {
  const int q = (int)(((float)i + 0.5f) * r.rcp);
  return slab_pos(r, q, i - q * r.rc);
}

// Eclipse terms are rare and spread over the orbit, so a wave whose lanes
// hold cadences all around it would run the out-of-line overlap area for a
// few lanes at almost every step.  Instead the eclipsing cadences are queued
// in LDS (slab position, separation, which star is in front) and applied 64
// at a time, every lane busy; the value written is the same v - term.
// Entries hold (dd with the sign of zz, slab position); entry kEclQ is the
// write target of the lanes that queue nothing (every lane stores, no
// exec-mask branch per cadence).
constexpr int kEclQ = 128;  // <= 63 carried + 64 appended (flushed after every chain's append)
__device__ __forceinline__ void ecl_apply(const WalkerConst& w, double* vals, const double* eq_dd,
                                          const int* eq_code, int first, int cnt, int lane) {
  if (lane < cnt) {
    const double q = eq_dd[first + lane];
    const double dR = sqrt(fabs(q)) * w.aR;  // projected separation [Rsun]
    vals[eq_code[first + lane]] -= eclipse_term(&w, dR, signbit(q) ? -1.0 : 1.0);  // out of line
  }
}

// Deferred cadence queue (HB_GQ = 1): the model pass writes every cadence's
// polynomial value to the slab and appends the cadences that need more to a
// per-wave region of global memory -- eclipsing ones (dd with the sign of zz,
// slab position) and the rare ones outside the fast sincos/fmod domain
// (cadence index, slab position | kSlowFlag).  After the pass, 64 entries at
// a time, the eclipse term (inlined) is subtracted from the slab value -- the
// same v - term as inline -- and slow-path cadences are recomputed in
// reference order.  The model loop then holds no function call: nothing of
// the loop's state is saved around one, and the out-of-line callee's
// register conventions no longer shape the loop's allocation.  Capacity per
// wave: 64 VPT entries (every cadence, worst case).
#ifndef HB_GQ
#define HB_GQ 1
#endif
constexpr int kSlowFlag = 1 << 30;
// One 16-B entry per queued cadence: (dd with the sign of zz, code = slab
// position | kSlowFlag for the slow path); one store, one load.
struct DeferQ {
  char* e;  // this wave's entries (the base is held in VGPRs: no SGPR spill reloads per push)
  int n;    // entries (wave-uniform)
};
// HB_DQ_SINK: the push is branch-free -- lanes that queue nothing store into
// the wave's sink entry (the 16 B in front of its region, never read), so the
// model pass's step stays one basic block that the scheduler can interleave
// (an exec-mask branch per push split it); 0: the branching push.
#ifndef HB_DQ_SINK
#define HB_DQ_SINK 1
#endif
constexpr int kDqSink = HB_DQ_SINK ? 1 : 0;  // entries in front of a wave's region
__device__ __forceinline__ void dq_push(DeferQ& q, bool push, double a, int code) {
  const unsigned long long bal = wave_ballot(push);
  // global address space spelled out (the VGPR base hides it from inference)
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(1))) d2v gdouble2;
  const uint32_t pos = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)bal, (unsigned)q.n));
  const d2v ent = {a, __longlong_as_double((long long)code)};
#if HB_DQ_SINK
  const long off = push ? (long)pos << 4 : -16L;
  *(gdouble2*)(q.e + off) = ent;
#else
  if (push) *(gdouble2*)(q.e + (size_t)(pos << 4)) = ent;
#endif
  q.n += __popcll(bal);
}
// t: the light curve's times in cadence order (slow-path entries: the cadence
// is recovered from the slab position, row = position / stride)
__device__ __forceinline__ void dq_apply(const WalkerConst& w, double* vals, const DeferQ& q,
                                         const double* __restrict__ t, const Rows& rw, int n, int lane) {
  if (q.n == 0) return;
  typedef __attribute__((address_space(1))) const double gcdouble;
  typedef __attribute__((address_space(1))) const long long gclong;
  const gcdouble* qa = (const gcdouble*)q.e;
  // the queue's stores are complete (acknowledged) before this wave reads them back
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  double a_n = 0.0;
  int c_n = 0;
  if (lane < q.n) {
    a_n = qa[2 * lane];
    c_n = (int)((const gclong*)qa)[2 * lane + 1];
  }
  for (int b = 0; b < q.n; b += 64) {  // wave-uniform
    const double a = a_n;
    const int code = c_n;
    const bool live = b + lane < q.n;
    const int i2 = b + 64 + lane;
    if (i2 < q.n) {  // the next batch's entries in flight while this one computes
      a_n = qa[2 * i2];
      c_n = (int)((const gclong*)qa)[2 * i2 + 1];
    }
    if (live) {
      if (code & kSlowFlag) {  // rare: reference-order path (eclipse included)
        const int sp = code & ~kSlowFlag;
        const int row = sp / rw.stride;
        const int cad = min(row * rw.rc + (sp - row * rw.stride), n - 1);
        vals[sp] = hb_cadence_flux_slow(t[cad], &w);
      } else {
        const double dR = sqrt_fast(fabs(a)) * w.aR;  // projected separation [Rsun]
        vals[code] -= eclipse_term_inl(&w, dR, signbit(a) ? -1.0 : 1.0);
      }
    }
  }
}

// Whether a walker's Kepler solves take the warm chains: e <= kWarmEmax (the
// reference's five steps converge, so the root is the same) and the first
// Newton correction after the first-order start, |d1| <= e dM^2 / (2 (1-e)^3)
// for the light curve's typical phase step dM (gap = 90th percentile of the
// cadence spacing, host-side), at most kWarmD1: the two-step fast path then
// holds for nearly every cadence.  Otherwise (high e, sparse or shuffled
// cadences) the cold path with four interleaved cadences per lane is faster.
#ifndef HB_WARM_D1
#define HB_WARM_D1 0x1p-10
#endif
#ifndef HB_CHAIN_VPT_MIN
#define HB_CHAIN_VPT_MIN 8
#endif
#ifndef HB_CHAIN_VPT_MAX
#define HB_CHAIN_VPT_MAX 32
#endif
__device__ __forceinline__ bool chain_eligible(const WalkerConst& w, double gap) {
  const double e = w.e;
  const double dm = gap * kDay * fabs(w.mA);
  const double ome = 1.0 - e;
  return (e <= kWarmEmax) && (e * dm * dm <= 2.0 * HB_WARM_D1 * ome * ome * ome);
}

// Wave pacing.  The waves sharing a SIMD are issued by priority, then age:
// with equal priorities the oldest wave runs nearly unimpeded and finishes
// first, and the youngest runs its last stretch alone, latency-bound
// (scripts/wave_clocks.py: finish times 46k/69k/89k/107k cycles for the four
// waves of a SIMD at C2).  A Pacer lowers a wave's priority as it gets ahead:
//   HB_PRIO == 1: by quartile of its own model pass (3 -> 0);
//   HB_PRIO == 2: by its lead over the slowest wave of its workgroup on the
//                 same SIMD (progress words in LDS, multi-walker workgroups).
struct Pacer {
  uint32_t* prog;  // WPB progress words (simd << 16 | progress/16), nullptr: none
  uint32_t tag;    // this wave's simd << 16
  int wib;         // wave in block
  int wpb;         // waves per block
  int lane;
  uint32_t inc;    // (16 << 8) / steps
  int q1, q2, q3;  // first steps of the 2nd, 3rd and 4th quarter
  __device__ __forceinline__ void begin(int steps) {
    inc = (16u << 8) / (uint32_t)(steps > 0 ? steps : 1);
    q1 = (steps + 3) >> 2;
    q2 = (steps + 1) >> 1;
    q3 = (3 * steps + 3) >> 2;
  }
  __device__ __forceinline__ void step(int j, int n) const {
#if HB_PRIO == 1
    (void)n;
    if (j == q1) __builtin_amdgcn_s_setprio(2);
    if (j == q2) __builtin_amdgcn_s_setprio(1);
    if (j == q3) __builtin_amdgcn_s_setprio(0);
#elif HB_PRIO == 2
    (void)n;
    if (prog == nullptr) return;
    const uint32_t p = ((uint32_t)j * inc) >> 8;
    if (lane == 0) prog[wib] = tag | p;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t v = lane < wpb ? prog[lane] : 0xffffffffu;
    uint32_t q = ((v & 0xffff0000u) == tag) ? (v & 0xffffu) : 0xffffu;
    q = min(q, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0xB1, 0xf, 0xf, false));
    q = min(q, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x4E, 0xf, 0xf, false));
    q = min(q, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x141, 0xf, 0xf, false));
    q = min(q, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x140, 0xf, 0xf, false));
    const uint32_t lead = p - (uint32_t)__builtin_amdgcn_readfirstlane((int)q);  // row 0 holds the min
    if (lead == 0) __builtin_amdgcn_s_setprio(3);
    else if (lead <= 2) __builtin_amdgcn_s_setprio(2);
    else if (lead <= 4) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#else
    (void)j;
    (void)n;
#endif
  }
};

// Virtual phase table (VT): the entry (sin, cos)(t DAY 2pi/P0) a walker on
// the table period (w.tab = 1: its Pc equals P0 bit for bit, so w.mA is
// 2pi/P0 computed the same way) would read, evaluated in place with the
// expression the prep writes the table with -- bit-identical, no table in
// memory (the catalog's fused launches, whose workgroups mix targets)
__device__ __forceinline__ double2 vt_entry(double t, const WalkerConst& w) {
  double sv, cv;
  sincos_table((t * kDay) * w.mA, sv, cv);
  return make_double2(sv, cv);
}

// Cold path in the one-wave kernel: the wave sweeps the light curve 64*K
// consecutive cadences at a time (cadence base + k*64 + lane), so the eclipse
// lanes of an iteration are neighbours in phase and the inline eclipse term
// runs only on the few iterations that cross an eclipse.  Values are stored
// at the lane-row slab positions (slab_pos_of) that the key load reads.
// NT threads per walker (64, or 128 for a pair of waves), thread tid
template <int NT = 64, bool VT = false>
__device__ __forceinline__ void model_pass_cold(const double* __restrict__ t, const double2* __restrict__ ph,
                                                int n, const Rows& rw, const WalkerConst& w, double* vals,
                                                int lane, Pacer pc, DeferQ& dq) {
  constexpr int K = HB_K;
  const bool vt = VT && ph == nullptr;                        // entries evaluated in place
  const bool tab = (vt || ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  const int last = n - 1;
  const int nit = (n + K * NT - 1) / (K * NT);
  pc.begin(nit);
  for (int base = 0, it = 0; base < n; base += K * NT, ++it) {
    pc.step(it, nit);
    double tk[K], v[K];
    double2 pk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = min(base + k * NT + lane, last);
      tk[k] = t[i];
      pk[k] = tab ? (vt ? vt_entry(tk[k], w) : ph[i]) : make_double2(0.0, 1.0);
    }
    bool bad;
#if HB_SPLIT_LIVE
    __asm__ volatile("" ::: "memory");
#endif
#if HB_GQ
    double dd[K], zz[K];
    hb_cadence_poly_k<K>(tk, pk, tab, w, v, dd, zz, bad);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = base + k * NT + lane;
      const int sp = slab_pos_of(rw, i);
      if (i < n) vals[sp] = v[k];
      const bool need = (!bad) & eclipse_lane(w, dd[k], zz[k]);
      dq_push(dq, (i < n) & (bad | need), copysign(dd[k], zz[k]), sp | (bad ? kSlowFlag : 0));
    }
#else
    hb_cadence_flux_k<K>(tk, pk, tab, w, v, bad);
    if (wave_any(bad)) {  // out-of-domain angles: reference-order ocml path
      if (bad) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = hb_cadence_flux_slow(tk[k], &w);
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = base + k * NT + lane;
      if (i < n) vals[slab_pos_of(rw, i)] = v[k];
    }
#endif
  }
}

// tT: the light curve's times in lane-row order (tT[c * 64 + l] = t[l * rc + c],
// build_rows), so the step-c loads of the 64 lanes are one coalesced 512-B
// request instead of 64 strided ones
// NR: lane rows of the walker (the arrays' pitch: 64, or 128 for a pair of
// waves, each passing tT offset by its first row); row: this lane's row
template <int VPT, int NR = 64>
__device__ __forceinline__ void model_pass_chain(const double* __restrict__ tT, const double2* __restrict__ ph,
                                                 int n, const Rows& rw, const WalkerConst& w, double* vals,
                                                 double* eq_dr, int* eq_code, int lane, int row, Pacer pc, DeferQ& dq
#ifdef HB_CLK_STEP0
                                                 , unsigned long long& clk_step0
#endif
                                                 ) {
  constexpr int KCM = NR > 64 ? HB_PAIR_KC : HB_KC;
  constexpr int KC = VPT < KCM ? VPT : KCM;
  const int lc = (rw.rc + KC - 1) / KC;  // chain length (wave-uniform)
  const bool tab = (ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  const int last = n - 1;
  const int base = row * rw.rc;
  const int rs = row * rw.stride, lsw = HB_ODD_STRIDE ? 0 : (row & rw.swz);  // slab_pos = rs + (c ^ lsw)
#if !HB_GQ
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  int qn = 0;  // queued eclipse cadences (wave-uniform)
#endif
  ChainState<KC> st;
  double tk[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) tk[k] = tT[min(k * lc, rw.rc - 1) * NR + lane];
  pc.begin(lc);
  for (int j = 0; j < lc; ++j) {
    pc.step(j, lc);
#ifdef HB_CLK_STEP0  // experiment builds only: the chains' cold first step ends here
    if (j == 1) clk_step0 = __builtin_amdgcn_s_memtime();
#endif
#if defined(HB_PAD_V) || defined(HB_PAD_S)  // experiment builds only: issue-cost probes
    {
      int x = j;
#ifdef HB_PAD_V
#pragma unroll
      for (int q = 0; q < HB_PAD_V; ++q) __asm__ volatile("v_add_u32 %0, 1, %0" : "+v"(x));
#endif
#ifdef HB_PAD_S
#pragma unroll
      for (int q = 0; q < HB_PAD_S; ++q) __asm__ volatile("s_add_u32 %0, %0, 1" : "+s"(x) :: "scc");
#endif
    }
#endif
    double tn[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) tn[k] = tT[min(k * lc + j + 1, rw.rc - 1) * NR + lane];
    double v[KC], dd[KC], zz[KC];
    bool bad;
#if HB_SPLIT_LIVE
    __asm__ volatile("" ::: "memory");
#endif
#if HB_ABLATE_MODEL  // experiment builds only: trivial model, same data flow
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      v[k] = tk[k] * w.kb + w.kr0;
      dd[k] = 1.0;
      zz[k] = 0.0;
    }
    bad = false;
#else
    if (j == 0) {  // the chains' first cadences: the reference's start (table entries)
      double2 p0[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) p0[k] = tab ? ph[min(base + k * lc, last)] : make_double2(0.0, 1.0);
      hb_cadence_flux_chain<KC>(tk, p0, tab, true, w, st, v, dd, zz, bad);
    } else {  // warm; a cadence that falls back to the reference start evaluates sin/cos directly
      const double2 p0[KC] = {};
      hb_cadence_flux_chain<KC>(tk, p0, false, false, w, st, v, dd, zz, bad);
    }
#endif
#if HB_GQ
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = k * lc + j;
      if (c < rw.rc) {  // wave-uniform: the last chain may run past the row end
        // cadences past n (the last row's padding) store harmless values: their keys are masked;
        // the rows kernel (NR > 128) sizes its slab to the live rows and stores no others
        const int sp = rs + (c ^ lsw);
        const bool live = NR <= 128 || row < rw.live;
        if (live) vals[sp] = v[k];
        const bool need = (!bad) & eclipse_lane(w, dd[k], zz[k]);
        dq_push(dq, live & (bad | need), copysign(dd[k], zz[k]), sp | (bad ? kSlowFlag : 0));
      }
      tk[k] = tn[k];
    }
#else
    if (wave_any(bad)) {  // out-of-domain angles: reference-order ocml path (eclipse included)
      if (bad) {
#pragma unroll
        for (int k = 0; k < KC; ++k) v[k] = hb_cadence_flux_slow(tk[k], &w);
      }
    }
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = k * lc + j;
      if (c < rw.rc) {  // wave-uniform: the last chain may run past the row end
        // cadences past n (the last row's padding) store harmless values: their keys are masked
        const int sp = rs + (c ^ lsw);
        vals[sp] = v[k];
#ifdef HB_ABLATE_ECL  // experiment builds only: no eclipse test
        const bool need = false;
#else
        const bool need = !bad && eclipse_lane(w, dd[k], zz[k]);
#endif
        const uint64_t bal = wave_ballot(need);
        const int pos = need ? qn + __popcll(bal & lt_mask) : kEclQ;
        eq_dr[pos] = copysign(dd[k], zz[k]);  // sign bit: which star is in front
        eq_code[pos] = sp;
        qn += __popcll(bal);
      }
      tk[k] = tn[k];
      const bool last = (j == lc - 1) && (k == KC - 1);
      while (qn >= 64 || (last && qn > 0)) {  // wave-uniform
        const int cnt = qn < 64 ? qn : 64;
        ecl_apply(w, vals, eq_dr, eq_code, qn - cnt, cnt, lane);
        qn -= cnt;
      }
    }
#endif
  }
}

// Software-pipelined model_pass_chain (HB_GQ; HB_CHAIN_SPLIT): the loop body
// of step j holds step j's warm Kepler solve and step j-1's polynomial, which
// both read only the chain state left by step j-1 -- one basic block with
// two independent dependency chains per Kepler chain (ILP 2 KC instead of KC
// for the latency-bound tail of the launch).  Step j-1's values are stored and
// queued after it, then step j is finished (converged lanes: the reciprocal;
// else the general Newton loop / the reference's start).  Values, queue
// entries and slab positions are those of model_pass_chain.
#ifndef HB_PIPE
#define HB_PIPE 1
#endif
// the walker constants are reloaded (scalar loads) at every pipelined step
// instead of being held in SGPRs across the loop: SGPR spills 138 -> 111
// (fused C2 kernel) and 206 -> 142 (device-sampler eval + Hastings), time
// unchanged (C2 41.38-41.43 vs 41.37-41.39 us per step, device loop 0.0925
// vs 0.0929 ms; profiles/r04/r04n_*.json)
#ifndef HB_PIPE_RELOAD
#define HB_PIPE_RELOAD 1
#endif
#ifndef HB_EMIT_LATE
#define HB_EMIT_LATE 1
#endif
#ifndef HB_POLY_PIN
#define HB_POLY_PIN 1
#endif
template <int VPT, int NR = 64, bool VT = false>
__device__ __forceinline__ void model_pass_chain_pipe(const double* __restrict__ tT, const double2* __restrict__ ph,
                                                      int n, const Rows& rw, const WalkerConst& w, double* vals,
                                                      int lane, int row, Pacer pc, DeferQ& dq) {
#if HB_CHAIN_SPLIT && HB_GQ
  constexpr int KCM = NR > 64 ? HB_PAIR_KC : HB_KC;
  constexpr int KC = VPT < KCM ? VPT : KCM;
  const int lc = (rw.rc + KC - 1) / KC;  // chain length (wave-uniform)
  const bool vt = VT && ph == nullptr;                        // entries evaluated in place
  const bool tab = (vt || ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  const int last = n - 1;
  const int base = row * rw.rc;
  const int rs = row * rw.stride, lsw = HB_ODD_STRIDE ? 0 : (row & rw.swz);  // slab_pos = rs + (c ^ lsw)
  const bool live = NR <= 128 || row < rw.live;
  ChainState<KC> st;
  double tk[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) tk[k] = tT[min(k * lc, rw.rc - 1) * NR + lane];
  // the step whose polynomial is pending: its (s, c, 1/den) are the chain state
  bool pend_ok = true;
  {  // step 0: the chains' first cadences (the reference's start, table entries)
    double2 p0[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
      p0[k] = tab ? (vt ? vt_entry(tk[k], w) : ph[min(base + k * lc, last)]) : make_double2(0.0, 1.0);
    chain_first<KC>(tk, p0, tab, w, st, pend_ok);
  }
  // store the pending step jp's values and queue its eclipse / slow-path cadences
  auto emit = [&](int jp, const double (&v)[KC], const double (&dd)[KC], const double (&zz)[KC], bool bad) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = k * lc + jp;
      if (c < rw.rc) {  // wave-uniform
        const int sp = rs + (c ^ lsw);
        if (live) vals[sp] = v[k];
        const bool need = (!bad) & eclipse_lane(w, dd[k], zz[k]);
        dq_push(dq, live & (bad | need), copysign(dd[k], zz[k]), sp | (bad ? kSlowFlag : 0));
      }
    }
  };
  const WarmK wk = warm_k(w.e);
  pc.begin(lc);
  for (int j = 1; j < lc; ++j) {
    pc.step(j, lc);
#if HB_PIPE_RELOAD
    __asm__ volatile("" ::: "memory");
#endif
#pragma unroll
    for (int k = 0; k < KC; ++k) tk[k] = tT[min(k * lc + j, rw.rc - 1) * NR + lane];
    double m[KC], E[KC], s[KC], c[KC], ys[KC], v[KC], dd[KC], zz[KC];
    bool ok = true, fine;
    chain_kepler_warm<KC>(tk, w, st, m, E, s, c, ys, fine, ok, wk);  // step j
    flux_poly_inv_k<KC>(st.s, st.c, st.inv, w, v, dd, zz);      // step j - 1, same block
#if HB_POLY_PIN
    // the polynomial's values are materialised here, beside step j's solve:
    // otherwise the compiler sinks them into emit's conditional blocks, after
    // the solve, and the two no longer interleave
#pragma unroll
    for (int k = 0; k < KC; ++k) __asm__ volatile("" : "+v"(v[k]), "+v"(dd[k]), "+v"(zz[k]));
#endif
#if HB_EMIT_LATE
    // step j - 1's stores and pushes after step j's finish: their branches
    // (the wave-uniform row test) then do not split the solve and polynomial
    const bool pbad = !pend_ok;
    chain_finish_warm<KC>(tk, w, wave_all(fine), fine, m, E, s, c, ys, ok, st);
    emit(j - 1, v, dd, zz, pbad);
#else
    emit(j - 1, v, dd, zz, !pend_ok);
    chain_finish_warm<KC>(tk, w, wave_all(fine), fine, m, E, s, c, ys, ok, st);
#endif
    pend_ok = ok;
  }
  {  // the last step's polynomial
    double v[KC], dd[KC], zz[KC];
    flux_poly_inv_k<KC>(st.s, st.c, st.inv, w, v, dd, zz);
    emit(lc - 1, v, dd, zz, !pend_ok);
  }
#else
  (void)tT; (void)ph; (void)n; (void)rw; (void)w; (void)vals; (void)lane; (void)row; (void)pc; (void)dq;
#endif
}

// k-th smallest (0-based) of vals[0..n) by radix select; every thread of the
// block gets the same answer.  kmin/kmax: block-wide min/max keys.
template <int NW>
__device__ double block_select(const double* vals, long n, long kth, uint64_t kmin, uint64_t kmax,
                               SelShared* sh) {
  constexpr int NT = 64 * NW;
  const int tid = threadIdx.x;
  if (kmin == kmax) return dval(kmin);
  int hi = 63 - __builtin_clzll(kmin ^ kmax);  // highest undetermined bit
  uint64_t mask = (hi == 63) ? 0ull : ~((2ull << hi) - 1ull);
  uint64_t prefix = kmin & mask;
  uint32_t kk = (uint32_t)kth;
  uint32_t cnt = 0;
  while (true) {
    const int width = hi + 1 < 8 ? hi + 1 : 8;
    const int shift = hi + 1 - width;
    const uint32_t dmask = (1u << width) - 1u;
    for (int b = tid; b < 256; b += NT) sh->hist[b] = 0u;
    __syncthreads();
    for (long i = tid; i < n; i += NT) {
      const uint64_t key = dkey(vals[i]);
      if ((key & mask) == prefix) atomicAdd(&sh->hist[(uint32_t)(key >> shift) & dmask], 1u);
    }
    __syncthreads();
    if (tid < 64) {
      const uint32_t c0 = sh->hist[4 * tid + 0], c1 = sh->hist[4 * tid + 1];
      const uint32_t c2 = sh->hist[4 * tid + 2], c3 = sh->hist[4 * tid + 3];
      const uint32_t s = c0 + c1 + c2 + c3;
      uint32_t incl = s;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off, 64);
        if (tid >= off) incl += o;
      }
      const uint32_t excl = incl - s;
      if (excl <= kk && kk < incl) {
        uint32_t before = excl;
        int bin = 4 * tid;
        uint32_t c = c0;
        if (kk >= before + c0) { before += c0; bin += 1; c = c1;
          if (kk >= before + c1) { before += c1; bin += 1; c = c2;
            if (kk >= before + c2) { before += c2; bin += 1; c = c3; } } }
        sh->bin = bin;
        sh->before = before;
        sh->cnt = c;
      }
    }
    __syncthreads();
    const uint32_t bin = (uint32_t)sh->bin;
    kk -= sh->before;
    cnt = sh->cnt;
    prefix |= (uint64_t)bin << shift;
    mask |= (uint64_t)dmask << shift;
    hi = shift - 1;
    if (cnt == 1 || hi < 0) break;
  }
  if (hi < 0) return dval(prefix);
  // unique survivor: fetch its full key
  for (long i = tid; i < n; i += NT) {
    const uint64_t key = dkey(vals[i]);
    if ((key & mask) == prefix) sh->ans = key;
  }
  __syncthreads();
  return dval(sh->ans);
}

template <int NW>
__device__ __forceinline__ void block_minmax(uint64_t& kmn, uint64_t& kmx, SelShared* sh) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  kmn = wave_min_u64(kmn);
  kmx = wave_max_u64(kmx);
  if (NW > 1) {
    if (lane == 0) { sh->red_min[wave] = kmn; sh->red_max[wave] = kmx; }
    __syncthreads();
    kmn = sh->red_min[0];
    kmx = sh->red_max[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) {
      kmn = sh->red_min[k] < kmn ? sh->red_min[k] : kmn;
      kmx = sh->red_max[k] > kmx ? sh->red_max[k] : kmx;
    }
  }
}

template <int NW>
__device__ __forceinline__ double block_sum(double v, SelShared* sh) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  v = wave_sum(v);
  if (NW > 1) {
    __syncthreads();
    if (lane == 0) sh->red_sum[wave] = v;
    __syncthreads();
    v = sh->red_sum[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) v += sh->red_sum[k];
  }
  return v;
}

// ---------------------------------------------------------------------------
// kernel 2: one workgroup per walker
// mode 0: logL[w];  mode 1: template[w][0..n)
// ---------------------------------------------------------------------------
template <int NW, bool LDS>
__global__ __launch_bounds__(64 * NW) void hb_eval_kernel(
    const double* __restrict__ t, const double2* __restrict__ ph, const double* __restrict__ f,
    const double* __restrict__ isg,
    long n, long kth, const WalkerConst* __restrict__ wcs, double* __restrict__ logl,
    double* __restrict__ tmpl_out, double* __restrict__ scratch, int mode) {
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  SelShared* sh = reinterpret_cast<SelShared*>(smem);
  const int tid = threadIdx.x;
  const int wv = blockIdx.x;
  double* vals = LDS ? reinterpret_cast<double*>(smem + sizeof(SelShared))
                     : scratch + (size_t)wv * (size_t)n;
  const WalkerConst& w = wcs[wv];
  // Roche overflow replaces chi^2 by 1e15 whatever the template is
  // (likelihood3.c:866-869): the logL needs no light curve (block-uniform exit)
  if (mode == 0 && w.roche != 0.0) {
    if (tid == 0) logl[wv] = -kBig / 2.0;
    return;
  }

  // 1. model flux for every cadence
  uint64_t kmn, kmx;
  model_pass<NT>(t, ph, (int)n, w, vals, tid, kmn, kmx);
  __syncthreads();
  block_minmax<NW>(kmn, kmx, sh);

  // 2. median (element of rank kth in ascending order)
#if HB_ABLATE_SELECT  // experiment builds only: no median selection
  const double med = dval(kmn);
#else
  const double med = block_select<NW>(vals, n, kth, kmn, kmx, sh);
#endif

  // 3. normalise, blend, chi^2
  const double blend = w.blend, one_m_blend = 1.0 - w.blend, tune = w.tune;
  if (mode == 1) {
    double* o = tmpl_out + (size_t)wv * (size_t)n;
    for (long i = tid; i < n; i += NT) {
      double m = (vals[i] - med) + 1.0;
      o[i] = (blend + m * one_m_blend) * tune;
    }
    return;
  }
  double acc = 0.0;
  for (long i = tid; i < n; i += NT) {
    double m = (vals[i] - med) + 1.0;
    m = (blend + m * one_m_blend) * tune;
    const double r = (m - f[i]) * isg[i];  // isg = 1/max(sigma, 1e-5), hb_create
    acc += r * r;
  }
  const double chi2 = block_sum<NW>(acc, sh);
  if (tid == 0) {
    double c = chi2 + w.chi2_extra;
    if (w.roche != 0.0) c = kBig;
    logl[wv] = -c / 2.0;
  }
}

// ---------------------------------------------------------------------------
// One-wave-per-walker path (N <= 64*VPT): keys in VGPRs, the LDS template slab
// reused as a histogram (11-bit first digit), exact rank among <= 64
// survivors.  kth is the 0-based rank of likelihood3.c:97-101.
// ---------------------------------------------------------------------------
#ifndef HB_SEL_BITS1
#define HB_SEL_BITS1 10
#endif
#ifndef HB_SEL_BITS2
#define HB_SEL_BITS2 8
#endif
constexpr int kSelBits = HB_SEL_BITS1;   // first digit (whole light curve)
constexpr int kSelBits2 = HB_SEL_BITS2;  // later digits (the survivors of one bin)
#ifndef HB_SEL_V
#define HB_SEL_V 3  // 3: leaner keys / select / chi^2 (below); 2: previous version; 1: shuffle-based select
#endif
#ifndef HB_CAND
#define HB_CAND 64
#endif
constexpr int kCandMax = HB_CAND;  // survivors ranked directly (<= 64: one per lane)
// slab bytes from which the fused launch keeps the survivors inside the slab
// (above the 2^kSelBits-bin histogram)
constexpr int kCandInSlab = (4 << kSelBits) + 8 * kCandMax;

template <int VPT>
__device__ double wave_select(const uint64_t (&key)[VPT], uint32_t kth, uint64_t kmin, uint64_t kmax,
                              uint32_t* hist, uint64_t* cand) {
  const int lane = threadIdx.x;
  if (kmin == kmax) return dval(kmin);
  int hi = 63 - __builtin_clzll(kmin ^ kmax);
  uint64_t mask = (hi == 63) ? 0ull : ~((2ull << hi) - 1ull);
  uint64_t prefix = kmin & mask;
  uint32_t kk = kth;
  uint32_t cnt = 0;
  int bits = kSelBits;
  while (true) {
    const int width = hi + 1 < bits ? hi + 1 : bits;
    bits = kSelBits2;
    const int shift = hi + 1 - width;
    const uint32_t nb = 1u << width, dm = nb - 1u;
    for (uint32_t b = lane; b < nb; b += 64) hist[b] = 0u;
    __syncthreads();
#pragma unroll
    for (int v = 0; v < VPT; ++v)
      if ((key[v] & mask) == prefix) atomicAdd(&hist[(uint32_t)(key[v] >> shift) & dm], 1u);
    __syncthreads();
    // every lane owns nb/64 consecutive bins (nb <= 2048 -> <= 32 = 8 x uint4)
    const uint32_t per = nb >= 64 ? nb / 64 : 1u;
    const uint32_t b0 = (uint32_t)lane * per;
    uint32_t g[8];  // per-group (4-bin) sums, compile-time indexed
    uint32_t local = 0;
    if (per >= 4) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        g[q] = 0;
        if ((uint32_t)q * 4 < per) {
          const uint4 h4 = *reinterpret_cast<const uint4*>(&hist[b0 + 4 * q]);
          g[q] = h4.x + h4.y + h4.z + h4.w;
        }
        local += g[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) g[q] = 0;
      for (uint32_t j = 0; j < per; ++j)
        if (b0 + j < nb) local += hist[b0 + j];
    }
    uint32_t incl = local;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    const uint32_t excl = incl - local;
    const unsigned long long own = wave_ballot(excl <= kk && kk < incl);
    const int owner = __ffsll((long long)own) - 1;
    uint32_t bin = 0, before = 0, c = 0;
    if (lane == owner) {
      before = excl;
      bin = b0;
      if (per >= 4) {  // pick the 4-bin group, then the bin: no dependent LDS chain
        uint32_t acc = excl;
        int grp = 0;
        bool stop = false;
#pragma unroll
        for (int q = 0; q < 7; ++q) {  // the rank lies in this lane: group <= 7
          stop |= !((uint32_t)(q + 1) * 4 < per && kk >= acc + g[q]);
          if (!stop) { acc += g[q]; grp = q + 1; }
        }
        const uint4 h4 = *reinterpret_cast<const uint4*>(&hist[b0 + 4 * grp]);
        before = acc;
        bin = b0 + 4 * grp;
        c = h4.x;
        if (kk >= before + c) { before += c; ++bin; c = h4.y;
          if (kk >= before + c) { before += c; ++bin; c = h4.z;
            if (kk >= before + c) { before += c; ++bin; c = h4.w; } } }
      } else {
        c = hist[bin];
        while (kk >= before + c) {
          before += c;
          ++bin;
          c = hist[bin];
        }
      }
    }
    bin = __shfl(bin, owner, 64);
    before = __shfl(before, owner, 64);
    cnt = __shfl(c, owner, 64);
    kk -= before;
    prefix |= (uint64_t)bin << shift;
    mask |= (uint64_t)dm << shift;
    hi = shift - 1;
    if (cnt <= (uint32_t)kCandMax || hi < 0) break;
    __syncthreads();  // histogram reads done before the next clear
  }
  if (hi < 0) return dval(prefix);
  // compact the cnt survivors, then rank them exactly
  uint32_t basec = 0;
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const bool m = (key[v] & mask) == prefix;
    const unsigned long long bal = wave_ballot(m);
    if (m) cand[basec + __popcll(bal & ((1ull << lane) - 1ull))] = key[v];
    basec += (uint32_t)__popcll(bal);
  }
  __syncthreads();
  const uint64_t mine = (uint32_t)lane < cnt ? cand[lane] : ~0ull;
  uint32_t r = 0;
  for (uint32_t j = 0; j < cnt; ++j) {
    const uint64_t o = cand[j];
    r += (o < mine) | ((o == mine) & (j < (uint32_t)lane));
  }
  const unsigned long long hit = wave_ballot((uint32_t)lane < cnt && r == kk);
  const int who = __ffsll((long long)hit) - 1;
  const uint64_t ans = __shfl(mine, who, 64);
  return dval(ans);
}

// ---------------------------------------------------------------------------
// Wave-level primitives without LDS round trips: DPP moves (GCN row_shr /
// row_bcast / quad_perm / mirrors) and v_readlane.  __shfl* lower to
// ds_bpermute, one LDS round trip per step; these stay in the VALU.
// ---------------------------------------------------------------------------
// inclusive prefix sum over the 64 lanes (all lanes active)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(v), l));
}

// Butterfly inside each row of 16 (xor 1, xor 2, half mirror, mirror: every
// lane of a row ends with the same row result, operands commuted only), then
// the four row results through v_readlane.  Op must be commutative.
template <class Op>
__device__ __forceinline__ uint64_t wave_reduce_u64(uint64_t v, Op op) {
  v = op(v, dpp_u64<0xB1>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_u64<0x4E>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_u64<0x141>(v));  // row_half_mirror
  v = op(v, dpp_u64<0x140>(v));  // row_mirror
  return op(op(readlane_u64(v, 0), readlane_u64(v, 16)), op(readlane_u64(v, 32), readlane_u64(v, 48)));
}
struct OpMinU64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a < b ? a : b; } };
struct OpMaxU64 { __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; } };
struct OpAddF64 {
  __device__ uint64_t operator()(uint64_t a, uint64_t b) const {
    return (uint64_t)__double_as_longlong(__longlong_as_double((long long)a) + __longlong_as_double((long long)b));
  }
};
__device__ __forceinline__ double wave_sum_dpp(double v) {
  return __longlong_as_double((long long)wave_reduce_u64((uint64_t)__double_as_longlong(v), OpAddF64()));
}

// Wave-level bin search over a 2^B-bin LDS histogram: the bin holding rank
// kk, the count before it and its count (uniform across the wave).  Every
// lane owns PER consecutive bins; DPP scan of the per-lane sums; the owning
// lane found by ballot walks its bins (group of 4, then bin) and v_readlane
// broadcasts the result.
template <int B>
__device__ __forceinline__ void wave_pick_bin(const uint32_t* hist, int lane, uint32_t kk, uint32_t& bin_out,
                                              uint32_t& before_out, uint32_t& cnt_out) {
  constexpr int PER = (1 << B) / 64;
  constexpr int Q = PER / 4;
  const uint4* h4 = reinterpret_cast<const uint4*>(hist);
  uint32_t h[PER];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const uint4 x = h4[lane * Q + q];
    h[4 * q] = x.x;
    h[4 * q + 1] = x.y;
    h[4 * q + 2] = x.z;
    h[4 * q + 3] = x.w;
  }
  uint32_t g[Q];
  uint32_t local = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    g[q] = h[4 * q] + h[4 * q + 1] + h[4 * q + 2] + h[4 * q + 3];
    local += g[q];
  }
  const uint32_t incl = wave_scan_incl(local);
  const uint32_t excl = incl - local;
  const unsigned long long own = wave_ballot(excl <= kk && kk < incl);
  const int owner = __builtin_amdgcn_readfirstlane(__ffsll((long long)own) - 1);
  // every lane walks its own bins (group of 4, then bin); the owner's is kept
  uint32_t before = excl;
  int grp = 0;
  bool go = true;
#pragma unroll
  for (int q = 0; q + 1 < Q; ++q) {
    go = go && (kk >= before + g[q]);
    if (go) { before += g[q]; grp = q + 1; }
  }
  uint32_t c0 = h[0], c1 = h[1], c2 = h[2], c3 = h[3];
#pragma unroll
  for (int q = 1; q < Q; ++q)
    if (grp == q) { c0 = h[4 * q]; c1 = h[4 * q + 1]; c2 = h[4 * q + 2]; c3 = h[4 * q + 3]; }
  uint32_t bin = (uint32_t)(lane * PER + 4 * grp), c = c0;
  if (kk >= before + c) { before += c; ++bin; c = c1;
    if (kk >= before + c) { before += c; ++bin; c = c2;
      if (kk >= before + c) { before += c; ++bin; c = c3; } } }
  bin_out = (uint32_t)__builtin_amdgcn_readlane((int)bin, owner);
  before_out = (uint32_t)__builtin_amdgcn_readlane((int)before, owner);
  cnt_out = (uint32_t)__builtin_amdgcn_readlane((int)c, owner);
}

// One radix pass with 2^B bins over the keys that match `prefix` under
// `mask`: histogram (LDS atomics), DPP scan of the per-lane bin sums, the
// owning lane found by ballot, its bin/offset/count read back by v_readlane.
template <int VPT, int B>
__device__ __forceinline__ void select_pass(const uint64_t (&key)[VPT], uint32_t* hist, int lane, int& hi,
                                            uint64_t& mask, uint64_t& prefix, uint32_t& kk, uint32_t& cnt) {
  static_assert(B >= 8 && B <= 11, "4..32 bins per lane");
  constexpr int PER = (1 << B) / 64;  // consecutive bins owned by a lane
  constexpr int Q = PER / 4;          // uint4 per lane
  const int width = hi + 1 < B ? hi + 1 : B;
  const int shift = hi + 1 - width;
  const uint32_t dm = (1u << width) - 1u;
  uint4* h4 = reinterpret_cast<uint4*>(hist);
#pragma unroll
  for (int q = 0; q < Q; ++q) h4[lane * Q + q] = make_uint4(0u, 0u, 0u, 0u);
  HB_WSYNC();
#pragma unroll
  for (int v = 0; v < VPT; ++v)
    if ((key[v] & mask) == prefix) atomicAdd(&hist[(uint32_t)(key[v] >> shift) & dm], 1u);
  HB_WSYNC();
  uint32_t bin, before;
  wave_pick_bin<B>(hist, lane, kk, bin, before, cnt);
  kk -= before;
  prefix |= (uint64_t)bin << shift;
  mask |= (uint64_t)dm << shift;
  hi = shift - 1;
  HB_WSYNC();  // histogram reads done before the next clear
}

template <int VPT>
__device__ __forceinline__ double wave_select2(const uint64_t (&key)[VPT], uint32_t kth, uint64_t kmin,
                                               uint64_t kmax, uint32_t* hist, uint64_t* cand) {
  const int lane = threadIdx.x & 63;
  if (kmin == kmax) return dval(kmin);
  int hi = 63 - __builtin_clzll(kmin ^ kmax);
  uint64_t mask = (hi == 63) ? 0ull : ~((2ull << hi) - 1ull);
  uint64_t prefix = kmin & mask;
  uint32_t kk = kth, cnt = 0;
  select_pass<VPT, kSelBits>(key, hist, lane, hi, mask, prefix, kk, cnt);
  while (cnt > (uint32_t)kCandMax && hi >= 0) select_pass<VPT, kSelBits2>(key, hist, lane, hi, mask, prefix, kk, cnt);
  if (hi < 0) return dval(prefix);
  // compact the cnt survivors, then rank them exactly
  uint32_t basec = 0;
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const bool m = (key[v] & mask) == prefix;
    const unsigned long long bal = wave_ballot(m);
    if (m) cand[basec + __popcll(bal & ((1ull << lane) - 1ull))] = key[v];
    basec += (uint32_t)__popcll(bal);
  }
  HB_WSYNC();
  const uint64_t mine = (uint32_t)lane < cnt ? cand[lane] : ~0ull;
  uint32_t r = 0;
  for (uint32_t j = 0; j < cnt; ++j) {
    const uint64_t o = cand[j];
    r += (o < mine) | ((o == mine) & (j < (uint32_t)lane));
  }
  const unsigned long long hit = wave_ballot((uint32_t)lane < cnt && r == kk);
  const int who = __builtin_amdgcn_readfirstlane(__ffsll((long long)hit) - 1);
  return dval(readlane_u64(mine, who));
}

// ---------------------------------------------------------------------------
// HB_SEL_V == 3: the same keys, median and chi^2 with fewer non-fp64
// instructions (bit-identical results):
//  * order keys in 3-4 VALU (okey/oval: a sign mask instead of compare+select);
//  * the select's bracket from the keys' high words (32-bit min/max, DPP): it
//    holds every live key, and only its common prefix is used;
//  * pass 1 needs no prefix test (every live key shares the bracket's prefix;
//    padding keys ~0 land in the top bin, above the k-th);
//  * digits by one shift of the high word (bfe) or a funnel shift (alignbit),
//    the prefix test of later passes on the high word when the prefix is there;
//  * a light curve that fills every lane row (n = 64 VPT: C2, C4) drops the
//    per-key liveness masks (a wave-uniform branch into a FULL instantiation).
// ---------------------------------------------------------------------------
#ifndef HB_SEL_V
#define HB_SEL_V 3
#endif
__device__ __forceinline__ uint64_t okey(double v) {  // == dkey(v)
  const uint32_t lo = (uint32_t)__double2loint(v), hi = (uint32_t)__double2hiint(v);
  const uint32_t m = (uint32_t)((int32_t)hi >> 31);
  return ((uint64_t)(hi ^ (m | 0x80000000u)) << 32) | (uint64_t)(lo ^ m);
}
__device__ __forceinline__ double oval(uint64_t k) {  // == dval(k)
  const uint32_t lo = (uint32_t)k, hi = (uint32_t)(k >> 32);
  uint32_t m;  // sign-extended top bit (asm: kept a shift, not a compare + selects)
  __asm__("v_ashrrev_i32 %0, 31, %1" : "=v"(m) : "v"(hi));
  return __hiloint2double((int)(hi ^ (~m | 0x80000000u)), (int)~(lo ^ m));
}
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce_u32(uint32_t v, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false));  // row_mirror
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return op(op(a, b), op(c, d));
}
struct OpMinU32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; } };
struct OpMaxU32 { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; } };

// Whether key k carries `prefix` in its bits >= pshift (the digits fixed so
// far), and its digit [shift, shift + width).  HT: pshift >= 32 (the test on
// the high word), HD: shift >= 32 (the digit in the high word); wave-uniform.
template <bool HT>
__device__ __forceinline__ bool key_match(uint64_t k, int pshift, uint64_t prefix) {
  if (HT) return ((uint32_t)(k >> 32) >> (pshift - 32)) == (uint32_t)(prefix >> pshift);
  return (k >> pshift) == (prefix >> pshift);
}
template <bool HD>
__device__ __forceinline__ uint32_t key_digit(uint64_t k, int shift, uint32_t dm) {
  if (HD) return ((uint32_t)(k >> 32) >> (shift - 32)) & dm;
  return __builtin_amdgcn_alignbit((uint32_t)(k >> 32), (uint32_t)k, (uint32_t)shift) & dm;
}
template <int VPT, bool TEST, bool HT, bool HD>
__device__ __forceinline__ void select3_hist(const uint64_t (&key)[VPT], uint32_t* hist, int pshift, uint64_t prefix,
                                             int shift, uint32_t dm, uint32_t dummy) {
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const uint32_t b = key_digit<HD>(key[v], shift, dm);
    atomicAdd(&hist[TEST ? (key_match<HT>(key[v], pshift, prefix) ? b : dummy) : b], 1u);
  }
}
// One radix pass of 2^B bins (TEST: later passes; pass 1 counts every key).
template <int VPT, int B, bool TEST>
__device__ __forceinline__ void select3_pass(const uint64_t (&key)[VPT], uint32_t* hist, int lane, int& hi,
                                             int& pshift, uint64_t& prefix, uint32_t& kk, uint32_t& cnt) {
  static_assert(!TEST || (4 << B) + 256 <= (4 << kSelBits), "the TEST pass dummies fit in the slab");
  constexpr int PER = (1 << B) / 64, Q = PER / 4;
  const int width = hi + 1 < B ? hi + 1 : B;
  const int shift = hi + 1 - width;
  const uint32_t dm = (1u << width) - 1u;
  uint4* h4 = reinterpret_cast<uint4*>(hist);
#pragma unroll
  for (int q = 0; q < Q; ++q) h4[lane * Q + q] = make_uint4(0u, 0u, 0u, 0u);
  HB_WSYNC();
  // the non-matching keys' bin in TEST passes: one per lane, past the 2^B bins
  // (one shared dummy would be a 64-way same-address atomic per key)
  const uint32_t dummy = (1u << B) + (uint32_t)lane;
  if (shift >= 32) select3_hist<VPT, TEST, true, true>(key, hist, pshift, prefix, shift, dm, dummy);
  else if (!TEST || pshift >= 32) select3_hist<VPT, TEST, true, false>(key, hist, pshift, prefix, shift, dm, dummy);
  else select3_hist<VPT, TEST, false, false>(key, hist, pshift, prefix, shift, dm, dummy);
  HB_WSYNC();
  uint32_t bin, before;
  wave_pick_bin<B>(hist, lane, kk, bin, before, cnt);
  kk -= before;
  prefix |= (uint64_t)bin << shift;
  pshift = shift;
  hi = shift - 1;
  HB_WSYNC();  // histogram reads done before the next clear
}
template <int VPT, bool HT>
__device__ __forceinline__ uint32_t select3_compact(const uint64_t (&key)[VPT], uint64_t* cand, int pshift,
                                                    uint64_t prefix) {
  uint32_t basec = 0;
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const bool m = key_match<HT>(key[v], pshift, prefix);
    const unsigned long long bal = wave_ballot(m);
    if (m) {  // exec-masked: a shared dummy slot would serialise the non-matching lanes' writes
      const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, basec));
      cand[pos] = key[v];
    }
    basec += (uint32_t)__popcll(bal);
  }
  return basec;
}
// k-th smallest key (0-based) over the wave; hmin/hmax: min / max high words
// of the live keys
template <int VPT>
__device__ __forceinline__ double wave_select3(const uint64_t (&key)[VPT], uint32_t kth, uint32_t hmin, uint32_t hmax,
                                               uint32_t* hist, uint64_t* cand) {
  const int lane = threadIdx.x & 63;
  const uint64_t kmin = (uint64_t)hmin << 32, kmax = ((uint64_t)hmax << 32) | 0xffffffffull;
  int hi = 63 - __builtin_clzll(kmin ^ kmax);  // >= 31
  uint64_t prefix = hi == 63 ? 0ull : (kmin & ~((2ull << hi) - 1ull));
  int pshift = hi + 1;
  uint32_t kk = kth, cnt = 0;
  select3_pass<VPT, kSelBits, false>(key, hist, lane, hi, pshift, prefix, kk, cnt);
  while (cnt > (uint32_t)kCandMax && hi >= 0) select3_pass<VPT, kSelBits2, true>(key, hist, lane, hi, pshift, prefix, kk, cnt);
  if (hi < 0) return oval(prefix);
  const uint32_t nc = pshift >= 32 ? select3_compact<VPT, true>(key, cand, pshift, prefix)
                                   : select3_compact<VPT, false>(key, cand, pshift, prefix);
  HB_WSYNC();
  const uint64_t mine = (uint32_t)lane < nc ? cand[lane] : ~0ull;
  uint32_t r = 0;
  for (uint32_t j = 0; j < nc; ++j) {
    const uint64_t o = cand[j];
    r += (o < mine) | ((o == mine) & (j < (uint32_t)lane));
  }
  const unsigned long long hit = wave_ballot((uint32_t)lane < nc && r == kk);
  const int who = __builtin_amdgcn_readfirstlane(__ffsll((long long)hit) - 1);
  return oval(readlane_u64(mine, who));
}
// ---------------------------------------------------------------------------
// A pair of waves per walker (WPW = 2: N = 1025..2048).  One wave per walker
// would need 32 cadences per lane, whose 17-KB slab leaves LDS for 9 waves per
// CU; two waves of 16 cadences per lane each hold half of the walker's rows.
// The model pass, the deferred eclipse terms and the key loads stay per wave
// (each lane owns its row); the select's histograms, the survivors and the
// chi^2 halves are shared through LDS with workgroup barriers.  Both waves
// run the same bin picks on the same histogram, so every decision is uniform
// over the pair.
// ---------------------------------------------------------------------------
constexpr int kMaxWPW = 16;
struct PairShared {
  uint32_t hmn[kMaxWPW], hmx[kMaxWPW];  // per wave: min / max key high words
  double chi[kMaxWPW];                  // per wave: chi^2 partial
  uint32_t ncand;                       // survivor counter
  uint32_t pad[3];
};
static_assert(sizeof(PairShared) % 16 == 0, "LDS carve must stay 16-B aligned");

template <int VPT, int B, bool TEST>
__device__ __forceinline__ void pair_pass(const uint64_t (&key)[VPT], uint32_t* hist, int lane, int& hi,
                                          int& pshift, uint64_t& prefix, uint32_t& kk, uint32_t& cnt) {
  static_assert(!TEST || (4 << B) + 256 <= (4 << kSelBits), "the TEST pass dummies fit in the slab");
  constexpr int PER = (1 << B) / 64, Q = PER / 4;
  const int width = hi + 1 < B ? hi + 1 : B;
  const int shift = hi + 1 - width;
  const uint32_t dm = (1u << width) - 1u;
  uint4* h4 = reinterpret_cast<uint4*>(hist);
  if (threadIdx.x < 64) {  // wave 0 clears, wave 1 waits at the barrier
#pragma unroll
    for (int q = 0; q < Q; ++q) h4[lane * Q + q] = make_uint4(0u, 0u, 0u, 0u);
  }
  __syncthreads();
  const uint32_t dummy = (1u << B) + (uint32_t)lane;
  if (shift >= 32) select3_hist<VPT, TEST, true, true>(key, hist, pshift, prefix, shift, dm, dummy);
  else if (!TEST || pshift >= 32) select3_hist<VPT, TEST, true, false>(key, hist, pshift, prefix, shift, dm, dummy);
  else select3_hist<VPT, TEST, false, false>(key, hist, pshift, prefix, shift, dm, dummy);
  __syncthreads();
  uint32_t bin, before;
  wave_pick_bin<B>(hist, lane, kk, bin, before, cnt);  // both waves: the same pick
  kk -= before;
  prefix |= (uint64_t)bin << shift;
  pshift = shift;
  hi = shift - 1;
  __syncthreads();  // histogram reads done before the next clear
}
template <int VPT, bool HT>
__device__ __forceinline__ void pair_compact(const uint64_t (&key)[VPT], uint64_t* cand, PairShared* ps, int pshift,
                                             uint64_t prefix) {
  uint32_t mine = 0;
#pragma unroll
  for (int v = 0; v < VPT; ++v) mine += key_match<HT>(key[v], pshift, prefix) ? 1u : 0u;
  uint32_t tot = mine;  // the wave's survivors, then one LDS atomic for its base
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) tot += (uint32_t)__shfl_xor((int)tot, off, 64);
  uint32_t basec = 0;
  if ((threadIdx.x & 63) == 0) basec = atomicAdd(&ps->ncand, tot);
  basec = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)basec, 0, 64));
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const bool m = key_match<HT>(key[v], pshift, prefix);
    const unsigned long long bal = wave_ballot(m);
    if (m) {
      const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, basec));
      cand[pos] = key[v];
    }
    basec += (uint32_t)__popcll(bal);
  }
}
// k-th smallest key (0-based) over the pair; hmin/hmax: the pair's min / max
// high words.  ps->ncand is zero on entry (set before the caller's barrier).
template <int VPT>
__device__ __forceinline__ double pair_select3(const uint64_t (&key)[VPT], uint32_t kth, uint32_t hmin, uint32_t hmax,
                                               uint32_t* hist, uint64_t* cand, PairShared* ps) {
  const int lane = threadIdx.x & 63;
  const uint64_t kmin = (uint64_t)hmin << 32, kmax = ((uint64_t)hmax << 32) | 0xffffffffull;
  int hi = 63 - __builtin_clzll(kmin ^ kmax);  // >= 31
  uint64_t prefix = hi == 63 ? 0ull : (kmin & ~((2ull << hi) - 1ull));
  int pshift = hi + 1;
  uint32_t kk = kth, cnt = 0;
  pair_pass<VPT, kSelBits, false>(key, hist, lane, hi, pshift, prefix, kk, cnt);
  while (cnt > (uint32_t)kCandMax && hi >= 0) pair_pass<VPT, kSelBits2, true>(key, hist, lane, hi, pshift, prefix, kk, cnt);
  if (hi < 0) return oval(prefix);
  if (pshift >= 32) pair_compact<VPT, true>(key, cand, ps, pshift, prefix);
  else pair_compact<VPT, false>(key, cand, ps, pshift, prefix);
  __syncthreads();
  const uint32_t nc = cnt;  // == ps->ncand
  const uint64_t mine = (uint32_t)lane < nc ? cand[lane] : ~0ull;
  uint32_t r = 0;
  for (uint32_t j = 0; j < nc; ++j) {
    const uint64_t o = cand[j];
    r += (o < mine) | ((o == mine) & (j < (uint32_t)lane));
  }
  const unsigned long long hit = wave_ballot((uint32_t)lane < nc && r == kk);
  const int who = __builtin_amdgcn_readfirstlane(__ffsll((long long)hit) - 1);
  return oval(readlane_u64(mine, who));
}

// keys of this lane's row (slot v: cadence lane rc + v; slots v >= lim are
// padding ~0) and the lane's min / max key high words over its live slots
template <int VPT, bool FULL>
__device__ __forceinline__ void load_keys3(const double* vals, const Rows& rw, int lane, int lim, uint64_t (&key)[VPT],
                                           uint32_t& hmn, uint32_t& hmx) {
  constexpr int kCh = VPT < 8 ? VPT : (VPT >= 32 ? 4 : 8);
  hmn = ~0u;
  hmx = 0u;
#pragma unroll
  for (int v0 = 0; v0 < VPT; v0 += kCh) {
    double x[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) x[u] = vals[slab_pos(rw, lane, FULL ? v0 + u : (v0 + u < rw.rc ? v0 + u : rw.rc - 1))];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int v = v0 + u;
      const uint64_t kv = okey(x[u]);
      const uint32_t h = (uint32_t)(kv >> 32);
      if (FULL) {
        key[v] = kv;
        hmn = h < hmn ? h : hmn;
        hmx = h > hmx ? h : hmx;
      } else {
        const bool act = v < lim;
        key[v] = act ? kv : ~0ull;
        hmn = (act && h < hmn) ? h : hmn;
        hmx = (act && h > hmx) ? h : hmx;
      }
    }
  }
}
// chi^2 partial of this lane (the reference's per-cadence operations,
// likelihood3.c:679-685 and :822-832) or, mode 1, the template values
template <int VPT, bool FULL, int NR = 64>
__device__ __forceinline__ double chi2_keys3(const uint64_t (&key)[VPT], double med, const WalkerConst& w,
                                             const double* __restrict__ fT, const double* __restrict__ iT,
                                             const Rows& rw, int lane, int lim) {
  constexpr int kCh = VPT < 8 ? VPT : (VPT >= 32 ? 4 : 8);
  const double blend = w.blend, one_m_blend = 1.0 - w.blend, tune = w.tune;
  double acc = 0.0;
#pragma unroll
  for (int v0 = 0; v0 < VPT; v0 += kCh) {
    double fv[kCh], iv[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {  // row block vc (wave-uniform) + lane: scalar base, lane offset
      const int vc = FULL ? v0 + u : (v0 + u < rw.rc ? v0 + u : rw.rc - 1);
      fv[u] = (fT + vc * NR)[lane];
      iv[u] = (iT + vc * NR)[lane];
    }
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int v = v0 + u;
      double m = (oval(key[v]) - med) + 1.0;
      m = (blend + m * one_m_blend) * tune;
      const double r = (m - fv[u]) * iv[u];
      if (FULL) acc += r * r;
      else acc += v < lim ? r * r : 0.0;
    }
  }
  return acc;
}

#ifndef HB_PHASE_TAB
#define HB_PHASE_TAB 1  // 0: every walker evaluates sin/cos of the Kepler start directly
#endif
#ifndef HB_RUN_AGG
#define HB_RUN_AGG 1  // block select: one LDS atomic per run of equal bins in a row of 16 lanes
#endif
#ifndef HB_BLOCK_KEYS
#define HB_BLOCK_KEYS 1  // 0: N > 2048 uses the LDS-walking block select (previous version)
#endif
// Key slot v of `lane` holds cadence lane*rc + v (its own row; v >= rc is
// padding).  A light curve is smooth, so 64 consecutive cadences mostly share
// one histogram bin and a wave's LDS atomic would serialise on one address;
// lane-owned rows give each atomic instruction 64 cadences spread over the
// whole light curve.
__device__ __forceinline__ int key_index(const Rows& r, int v, int lane) { return lane * r.rc + v; }
__device__ __forceinline__ bool key_live(const Rows& r, int v, int lane, long n) {
  return (v < r.rc) & (lane * r.rc + v < n);
}

// ---------------------------------------------------------------------------
// Fused launch (PRE): the per-walker records of the workgroup's WPB walkers in
// the eval kernel's prologue, instead of a separate hb_prep_kernel launch.
// Waves 0-3 run the four prep roles with lane = walker (hb_prep.hpp, the
// same operations as hb_prep_kernel: bit-identical records); the other waves
// meanwhile fill the shared-period phase table into LDS (every workgroup the
// whole table, the values hb_prep_kernel writes: (sin, cos)(t_i DAY 2pi/P0)
// for walker 0's period P0) and store their workgroup's slice of it to the
// context's global table, so later launches (hb_evaluate_dev, the device
// sampler) see what a prep launch would have left.  The records go to the
// context's workspace too, where each eval wave reads its own with scalar
// loads after the prologue's last barrier (stores complete first).  The prep
// scratch aliases the waves' slabs, which the model pass only writes after
// that barrier.
// ---------------------------------------------------------------------------
template <int WPB, bool MULTI>
__device__ __forceinline__ void fused_prologue(const PreArgs& pa, int count, int n, const double* __restrict__ t,
                                               unsigned char* smem_all, double2* tabl) {
  static_assert(WPB >= kPrepRoles && WPB <= 16, "four prep roles, <= 1024 threads");
  constexpr int NT = 64 * WPB;
  PrepShared<WPB>& L = *reinterpret_cast<PrepShared<WPB>*>(smem_all);
  // catalog: the workgroup's walkers and their targets (past the prep scratch)
  double* mg = reinterpret_cast<double*>(smem_all + sizeof(PrepShared<WPB>));  // [3][WPB] magnitude data
  int* wl = reinterpret_cast<int*>(mg + 3 * WPB);
  int* wtl = wl + WPB;
  const int tid = threadIdx.x;
  HB_PCLK(0, 0);
  const int base = blockIdx.x * WPB;
  const int nb = min(WPB, count - base);
  if constexpr (MULTI) {
    if (tid < WPB) {
      const int wk = tid < nb ? pa.list[base + tid] : 0;
      const int tg = pa.wt[wk];
      wl[tid] = wk;
      wtl[tid] = tg;
      const TargetDesc& td = pa.tab[tg];
      mg[tid] = td.dist;
      mg[WPB + tid] = td.gmag;
      mg[2 * WPB + tid] = td.gerr;
    }
    __syncthreads();
  }
  {  // parameters, all loads in flight before the first LDS write
    constexpr int U = (WPB * kNpars + NT - 1) / NT;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      if constexpr (MULTI) {
        const int j = i / kNpars;
        v[u] = i < nb * kNpars ? pa.params[(size_t)wl[j] * kNpars + (i - j * kNpars)] : 0.0;
      } else {
        v[u] = i < nb * kNpars ? pa.params[(size_t)base * kNpars + i] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      if (i < nb * kNpars) L.sp[i] = v[u];
    }
  }
  // the table period: walker 0's (hb_prep_kernel's tab_pc of a single
  // context), or the first walker's of the walker's target (catalog)
  const double Pc0 = MULTI ? 0.0 : exp10(pa.params[2]) * kDay;
  auto tab_pc = [&](int j) -> double {
    if constexpr (MULTI) return exp10(pa.params[(size_t)pa.w0[wtl[j]] * kNpars + 2]) * kDay;
    return Pc0;
  };
  // (sin, cos)(t_i DAY 2pi/Pc0) for i = first, first + stride, ... < n, into
  // LDS; this workgroup's slice [lo, hi) of the cadences also to the global table
  auto table = [&](int first, int stride) {
    const double mA0 = kTwoPi / Pc0;
    const int G = (int)gridDim.x;
    const int lo = (int)((long)n * blockIdx.x / G), hi = (int)((long)n * (blockIdx.x + 1) / G);
    for (int i = first; i < n; i += stride) {
      double sv, cv;
      sincos_table((t[i] * kDay) * mA0, sv, cv);
      const double2 e = make_double2(sv, cv);
      tabl[i] = e;
      if (i >= lo && i < hi) pa.ph[i] = e;
    }
    if (blockIdx.x == 0 && first == 0 && pa.tab_pc != nullptr) *pa.tab_pc = Pc0;
  };
  __syncthreads();
  HB_PCLK(1, 0);
  auto none = []() {};
  if constexpr (MULTI) {  // no table: the eval waves evaluate its entries in place
    prep_records<WPB>(L, nb, pa.ma, nullptr, nullptr, 0, tab_pc, none, PrepNoIdle(), mg);
  } else if constexpr (WPB > kPrepRoles) {
    auto idle = [&]() {
      table(tid - 64 * kPrepRoles, NT - 64 * kPrepRoles);
      HB_PCLK(4, 64 * kPrepRoles);
    };
    prep_records<WPB>(L, nb, pa.ma, nullptr, nullptr, base, tab_pc, none, idle);
  } else {
    prep_records<WPB>(L, nb, pa.ma, nullptr, nullptr, base, tab_pc, none);
    table(tid, NT);  // four waves: the table after the roles
  }
  HB_PCLK(2, 0);
  {  // the records to the workspace (coalesced rows), complete before the barrier
    constexpr int U = (WPB * kWcDoubles + NT - 1) / NT;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      const int jw = i / kWcDoubles;  // record rows of kSoStride doubles in LDS
      v[u] = i < nb * kWcDoubles ? L.so[jw * kSoStride + (i - jw * kWcDoubles)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      if (i < nb * kWcDoubles) {
        if constexpr (MULTI) {
          const int j = i / kWcDoubles;
          reinterpret_cast<double*>(pa.wc)[(size_t)wl[j] * kWcDoubles + (i - j * kWcDoubles)] = v[u];
        } else {
          reinterpret_cast<double*>(pa.wc)[(size_t)base * kWcDoubles + i] = v[u];
        }
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // the stores acknowledged (L2) before any wave's scalar loads
  __syncthreads();
  HB_PCLK(3, 0);
}

// MULTI (catalog mode): the walker is list[blockIdx.x] and its light curve is
// its target's slice (tab[wt[walker]]); n and kth come from the descriptor.
// ACC (device sampler): the wave then runs the Hastings test and history write
// of its slot (hb_accept.hpp) on the logL it just computed, in place of a
// separate ds_accept launch.
// WPB > 1: WPB walkers (one wave each) per workgroup; a wave's LDS is its
// lds_per-byte slice.  The waves only meet at the progress-word barrier of
// the pacer (HB_PRIO == 2); everything else syncs per wave (HB_WSYNC).
// WPW = 2: a pair of waves per walker (N = 1025..2048, see PairShared): wave h
// owns lane rows 64 h .. 64 h + 63 of 128; VPT is then the cadences per lane
// of the pair's rows (<= 16).
// PRE: the fused launch (fused_prologue above): WPB walkers per workgroup, the
// records computed in the prologue, the phase table read from LDS.
template <int VPT, bool MULTI, bool ACC = false, int WPB = 1, int WPW = 1, bool PRE = false>
__global__ __launch_bounds__(64 * WPB * WPW) HB_WPE_ATTR void hb_eval_wave_kernel(
    const double* __restrict__ t, const double2* __restrict__ ph, const double* __restrict__ f,
    const double* __restrict__ isg, const double* __restrict__ rows,
    long n, long kth, const WalkerConst* __restrict__ wcs, double* __restrict__ logl,
    double* __restrict__ tmpl_out, int mode, int slab_bytes, double gap, const TargetDesc* __restrict__ tab,
    const int* __restrict__ wt, const int* __restrict__ list, hbds::AccArgs hst, int count, int lds_per,
    double* __restrict__ dqbuf, PreArgs pre) {
  static_assert(WPW == 1 || (WPW <= kMaxWPW && WPB == 1 && !ACC && HB_SEL_V == 3 && HB_GQ), "pair/rows: plain batched path");
  static_assert(!PRE || (WPW == 1 && !ACC && WPB >= kPrepRoles && HB_SEL_V == 3 && HB_GQ && HB_PRIO != 2),
                "fused launch: plain one-wave batched path");
  // catalog launches without a table (ph == nullptr: the fused launches, whose
  // workgroups mix targets, and the classes beside them, whose records launch
  // writes no tables) evaluate the per-target entries in place (vt_entry);
  // with the tables of the catalog's records launch they read them
  constexpr bool kVT = MULTI;
  static_assert(!kVT || (HB_PIPE && HB_CHAIN_SPLIT), "the virtual table needs the pipelined chain pass");
  constexpr int NR = 64 * WPW;  // lane rows per walker
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_all[];
  const int lane = threadIdx.x & 63;
  const int h = WPW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;  // wave of the pair
  const int row = h * 64 + lane;
  const int wib = WPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int slot = (int)blockIdx.x * WPB + wib;
  const bool valid = WPB == 1 || slot < count;
  unsigned char* smem = smem_all + (size_t)wib * (size_t)lds_per;
  if constexpr (PRE) {
    double2* tabl = reinterpret_cast<double2*>(smem_all + (size_t)WPB * (size_t)lds_per);
    fused_prologue<WPB, MULTI>(pre, count, (int)n, t, smem_all, tabl);
    // the records just written: scalar loads (constant address space), issued
    // only after the prologue's last barrier (the pointer passes through asm)
    typedef const __attribute__((address_space(4))) WalkerConst cwc_t;
    uint64_t a = (uint64_t)pre.wc;
    __asm__ volatile("" : "+s"(a));
    wcs = (const WalkerConst*)(cwc_t*)a;
    ph = tabl;
  }
  int wv = slot;
  if (ACC && hst.ecnt != nullptr && valid) wv = hbds::eval_slot_by_e(hst, slot, lane);  // device sampler
  if (MULTI && valid) {
    wv = list[slot];
    const TargetDesc& td = tab[wt[wv]];
    t += td.off;
    if (ph) ph += td.off;
    f += td.off;
    isg += td.off;
    rows += td.roff;
    n = td.n;
    kth = td.kth;
  }
  HB_CLK_BEGIN();
#if HB_PRIO
  __builtin_amdgcn_s_setprio(3);
#endif
  double* vals = reinterpret_cast<double*>(smem);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  // the select's survivors: past the slab, or (fused launch) inside it, past
  // the histogram (the slab is dead once the keys are in registers)
  uint64_t* cand = reinterpret_cast<uint64_t*>(smem + (PRE && slab_bytes >= kCandInSlab ? (4 << kSelBits) : slab_bytes));
  const WalkerConst& w = wcs[valid ? wv : 0];
#ifdef HB_ABLATE_EXIT  // experiment builds only: every wave takes the early exit (launch floor)
  const bool roche_exit = mode == 0;
#else
  const bool roche_exit = mode == 0 && w.roche != 0.0;
#endif
  Pacer pc{nullptr, 0u, wib, WPB, lane, 0u, 0, 0, 0};
#if HB_PRIO == 2
  if (WPB > 1) {
    // progress words: simd << 16 | progress; finished or idle waves report 0xffff
    uint32_t* prog = reinterpret_cast<uint32_t*>(smem_all + (size_t)WPB * (size_t)lds_per);
    const uint32_t simd = ((uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;  // HW_ID.simd_id
    pc.prog = prog;
    pc.tag = simd << 16;
    if (lane == 0) prog[wib] = pc.tag | ((valid && !roche_exit) ? 0u : 0xffffu);
    __syncthreads();  // the workgroup's only barrier
  }
#endif
  if (!valid) return;
  // the Hastings test's operands are loaded now, not after the likelihood
  // HB_ACC_PRE 1: all of it (uniform values and the 21-coordinate rows);
  // 2: the uniform values only, the rows when the test runs; 0: nothing
  hbds::AccPre apre{};
  if (ACC && HB_ACC_PRE == 1) apre = hbds::accept_prefetch(hst, wv, lane);
  if (ACC && HB_ACC_PRE == 2) apre = hbds::accept_prefetch_uniform(hst, wv);
  auto acc_tail = [&](double ly) {
    if (HB_ACC_PRE == 0) apre = hbds::accept_prefetch(hst, wv, lane);
    if (HB_ACC_PRE == 2) hbds::accept_prefetch_rows(hst, wv, lane, apre);
    const bool took = hbds::accept_slot_wave_pre(hst, wv, ly, lane, apre);
#if HB_SWAP_TAIL
    if (hst.tcnt != nullptr)  // tempering swaps (hb_accept.hpp), on the logL the test left in the slot
      hbds::swap_tail_wave(hst, wv, took ? ly : apre.lx, lane, smem);
#else
    (void)took;
#endif
  };
  if (roche_exit) {  // likelihood3.c:866-869, see hb_eval_kernel
    if (row == 0) logl[wv] = -kBig / 2.0;
    if (ACC) acc_tail(-kBig / 2.0);
    HB_CLK_END(wv);
    return;
  }

  uint64_t kmn, kmx;
  uint64_t key[VPT];
  const Rows rw = make_rows((int)n, NR);
  // t, f and 1/sigma in lane-row order (pitch NR), from this wave's first row
  const double* __restrict__ tT = rows + h * 64;
  const double* __restrict__ fT = rows + NR * rw.rc + h * 64;
  const double* __restrict__ iT = rows + 2 * NR * rw.rc + h * 64;
  PairShared* ps = reinterpret_cast<PairShared*>(smem + slab_bytes + 8 * kCandMax);  // WPW == 2 only
  DeferQ dq{nullptr, 0};
  if (HB_GQ) {  // this wave's region of the deferred queue (64 VPT entries of 16 B)
    dq.e = reinterpret_cast<char*>(dqbuf) + ((size_t)slot * WPW + (size_t)h) * (size_t)((64 * VPT + kDqSink) * 16) +
           kDqSink * 16;
    __asm__ volatile("" : "+v"(dq.e));  // a VGPR pair, not one more scalar to spill
  }
  {
    if (VPT >= HB_CHAIN_VPT_MIN && VPT <= HB_CHAIN_VPT_MAX && chain_eligible(w, MULTI ? tab[wt[wv]].gap : gap)) {
      // the eclipse queue shares the select's candidate area (dead until the select)
      double* eq_dr = reinterpret_cast<double*>(smem + slab_bytes);
      int* eq_code = reinterpret_cast<int*>(eq_dr + kEclQ + 1);
#if HB_PIPE && HB_CHAIN_SPLIT && HB_GQ && !defined(HB_CLK_STEP0) && !HB_ABLATE_MODEL
      (void)eq_dr;
      (void)eq_code;
      model_pass_chain_pipe<VPT, NR, kVT>(tT, ph, (int)n, rw, w, vals, lane, row, pc, dq);
#else
      model_pass_chain<VPT, NR>(tT, ph, (int)n, rw, w, vals, eq_dr, eq_code, lane, row, pc, dq
#ifdef HB_CLK_STEP0
                            , clkm_[3]
#endif
                            );
#endif
    } else {
      model_pass_cold<NR, kVT>(t, ph, (int)n, rw, w, vals, row, pc, dq);
    }
  }
#if HB_GQ
#ifndef HB_CLK_STEP0
  HB_CLK_MARK(3);
#endif
  HB_WSYNC();  // the slab values of every lane are in place
  // a pair's cold pass writes cadences of either wave's rows, and its queued
  // eclipse terms land there too: the pair meets before and after them
  if (WPW > 1) __syncthreads();
  dq_apply(w, vals, dq, t, rw, (int)n, lane);
  if (WPW > 1) __syncthreads();
#endif
  HB_CLK_MARK(0);
#if HB_PRIO == 2
  if (pc.prog != nullptr) {
    if (lane == 0) pc.prog[wib] = pc.tag | 0xffffu;  // model pass done: stop holding the others back
    __builtin_amdgcn_s_setprio(0);
  }
#endif
  HB_WSYNC();
#if HB_SEL_V == 3
  {
    // live key slots of this lane; a light curve of 64 VPT cadences fills every row
    const int lim = min(rw.rc, max(0, (int)n - row * rw.rc));
    const bool full = (rw.rc == VPT) && (n == (long)NR * VPT);  // wave-uniform
    uint32_t hmn, hmx;
    if (full) load_keys3<VPT, true>(vals, rw, row, lim, key, hmn, hmx);
    else load_keys3<VPT, false>(vals, rw, row, lim, key, hmn, hmx);
    hmn = wave_reduce_u32(hmn, OpMinU32());
    hmx = wave_reduce_u32(hmx, OpMaxU32());
    if (WPW > 1) {  // the walker's bracket; every wave's keys are loaded before the slab turns histogram
      if (lane == 0) {
        ps->hmn[h] = hmn;
        ps->hmx[h] = hmx;
        if (h == 0) ps->ncand = 0u;
      }
      __syncthreads();
      hmn = ps->hmn[0];
      hmx = ps->hmx[0];
#pragma unroll
      for (int q = 1; q < WPW; ++q) {
        hmn = min(hmn, ps->hmn[q]);
        hmx = max(hmx, ps->hmx[q]);
      }
    }
    HB_CLK_MARK(1);
    HB_WSYNC();  // the slab becomes the histogram
    const double med = WPW > 1 ? pair_select3<VPT>(key, (uint32_t)kth, hmn, hmx, hist, cand, ps)
                               : wave_select3<VPT>(key, (uint32_t)kth, hmn, hmx, hist, cand);
    HB_CLK_MARK(2);
    if (mode == 1) {
      const double blend = w.blend, one_m_blend = 1.0 - w.blend, tune = w.tune;
      double* o = tmpl_out + (size_t)wv * (size_t)n;
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        if (v < lim) {
          const double m = (oval(key[v]) - med) + 1.0;
          o[key_index(rw, v, row)] = (blend + m * one_m_blend) * tune;
        }
      }
      HB_CLK_END(wv);
      return;
    }
    const double acc = full ? chi2_keys3<VPT, true, NR>(key, med, w, fT, iT, rw, lane, lim)
                            : chi2_keys3<VPT, false, NR>(key, med, w, fT, iT, rw, lane, lim);
    double chi2 = wave_sum_dpp(acc);
    if (WPW > 1) {  // the waves' partials in a fixed order
      if (lane == 0) ps->chi[h] = chi2;
      __syncthreads();
      chi2 = ps->chi[0];
#pragma unroll
      for (int q = 1; q < WPW; ++q) chi2 += ps->chi[q];
    }
    double c = chi2 + w.chi2_extra;
    if (w.roche != 0.0) c = kBig;
    if (row == 0) logl[wv] = -c / 2.0;
    if (ACC) acc_tail(-c / 2.0);  // c is wave-uniform (readlanes)
    HB_CLK_END(wv);
    return;
  }
#endif
  // keys, and the lane's min/max keys.  Every slot is loaded unconditionally
  // (slot v >= rc reads row position rc - 1) so the VPT LDS reads are in
  // flight together, then masked; min/max run on the order keys (exact
  // bracket, NaN keys included, no IEEE min/max canonicalisation).
  constexpr int kCh = VPT < 8 ? VPT : (VPT >= 32 ? 4 : 8);  // slots per batch of loads in flight
  kmn = ~0ull;
  kmx = 0ull;
#pragma unroll
  for (int v0 = 0; v0 < VPT; v0 += kCh) {
    double x[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) x[u] = vals[slab_pos(rw, lane, v0 + u < rw.rc ? v0 + u : rw.rc - 1)];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int v = v0 + u;
      const bool act = key_live(rw, v, lane, n);
      const uint64_t kv = dkey(x[u]);
      key[v] = act ? kv : ~0ull;  // padding sorts last, never selected
      kmn = key[v] < kmn ? key[v] : kmn;
      kmx = (act && kv > kmx) ? kv : kmx;
    }
  }
#if HB_SEL_V == 1
  kmn = wave_min_u64(kmn);
  kmx = wave_max_u64(kmx);
#else
  kmn = wave_reduce_u64(kmn, OpMinU64());
  kmx = wave_reduce_u64(kmx, OpMaxU64());
#endif
  HB_CLK_MARK(1);
  HB_WSYNC();  // the slab becomes the histogram
#if HB_ABLATE_SELECT
  const double med = dval(kmn);
#else
#if HB_SEL_V == 1
  const double med = wave_select<VPT>(key, (uint32_t)kth, kmn, kmx, hist, cand);
#else
  const double med = wave_select2<VPT>(key, (uint32_t)kth, kmn, kmx, hist, cand);
#endif
#endif

  HB_CLK_MARK(2);
  const double blend = w.blend, one_m_blend = 1.0 - w.blend, tune = w.tune;
  if (mode == 1) {
    double* o = tmpl_out + (size_t)wv * (size_t)n;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      const int i = key_index(rw, v, lane);
      if (key_live(rw, v, lane, n)) {
        const double m = (dval(key[v]) - med) + 1.0;
        o[i] = (blend + m * one_m_blend) * tune;
      }
    }
    HB_CLK_END(wv);
    return;
  }
  // chi^2 operands in lane-row order (coalesced), loaded unconditionally
  // (slot v >= rc re-reads row rc - 1) so the loads are in flight together
  double acc = 0.0;
#pragma unroll
  for (int v0 = 0; v0 < VPT; v0 += kCh) {
    double fv[kCh], iv[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int vc = v0 + u < rw.rc ? v0 + u : rw.rc - 1;
      fv[u] = fT[vc * 64 + lane];
      iv[u] = iT[vc * 64 + lane];
    }
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int v = v0 + u;
      double m = (dval(key[v]) - med) + 1.0;
      m = (blend + m * one_m_blend) * tune;
      const double r = (m - fv[u]) * iv[u];
      acc += key_live(rw, v, lane, n) ? r * r : 0.0;
    }
  }
#if HB_SEL_V == 1
  const double chi2 = wave_sum(acc);
#else
  const double chi2 = wave_sum_dpp(acc);
#endif
  if (lane == 0) {
    double c = chi2 + w.chi2_extra;
    if (w.roche != 0.0) c = kBig;
    logl[wv] = -c / 2.0;
  }
  if (ACC) {
    double c = chi2 + w.chi2_extra;  // wave-uniform (the DPP sum ends in readlanes)
    if (w.roche != 0.0) c = kBig;
    acc_tail(__shfl(-c / 2.0, 0));
  }
  HB_CLK_END(wv);
}

// ---------------------------------------------------------------------------
// NW waves per walker with register keys (2048 < N <= 64*NW*VPT; config C3,
// N = 20 000).  Like the one-wave kernel, the LDS slab holds the model values
// only until every thread has its VPT order keys (cadence v*NT + tid: the
// chi^2 operands stay coalesced); the slab then carries the histogram.  Each
// radix pass is one LDS histogram of the block's survivors, scanned by wave 0
// (wave_pick_bin: DPP scan + readlane) and broadcast through SelShared.  The
// <= 64 survivors are appended (order free: equal keys are equal values) and
// ranked by wave 0.  Min/max and chi^2 reduce per wave by DPP, across waves
// through SelShared in wave order (deterministic).
// ---------------------------------------------------------------------------
template <int NW, int VPT, int B>
__device__ __forceinline__ void block_select_pass(const uint64_t (&key)[VPT], uint32_t* hist, SelShared* sh,
                                                  int tid, int& hi, uint64_t& mask, uint64_t& prefix,
                                                  uint32_t& kk, uint32_t& cnt) {
  constexpr int NT = 64 * NW, NB = 1 << B;
  const int width = hi + 1 < B ? hi + 1 : B;
  const int shift = hi + 1 - width;
  const uint32_t dm = (1u << width) - 1u;
  uint4* h4 = reinterpret_cast<uint4*>(hist);
  for (int q = tid; q < NB / 4; q += NT) h4[q] = make_uint4(0u, 0u, 0u, 0u);
  __syncthreads();
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
#if HB_RUN_AGG
    // neighbouring cadences mostly share a bin: add each run of equal bins
    // (within a row of 16 lanes: DPP row_shr:1 compares with lane-1) once,
    // from its first lane, instead of up to 64 same-address LDS atomics
    const bool m = (key[v] & mask) == prefix;
    const uint32_t b = m ? ((uint32_t)(key[v] >> shift) & dm) : 0xffffffffu;
    const uint32_t bp = (uint32_t)__builtin_amdgcn_update_dpp((int)0xfffffffeu, (int)b, 0x111, 0xf, 0xf, false);
    const bool head = m && (b != bp);
    const unsigned long long bound = wave_ballot(head || !m);  // lanes that start a run or hold no key
    if (head) {
      const int lane = tid & 63;
      const unsigned long long after = lane < 63 ? (bound >> (lane + 1)) : 0ull;
      const uint32_t len = after ? (uint32_t)__builtin_ctzll(after) + 1u : (uint32_t)(64 - lane);
      atomicAdd(&hist[b], len);
    }
#else
    if ((key[v] & mask) == prefix) atomicAdd(&hist[(uint32_t)(key[v] >> shift) & dm], 1u);
#endif
  }
  __syncthreads();
  if (tid < 64) {
    uint32_t bin, before, c;
    wave_pick_bin<B>(hist, tid, kk, bin, before, c);
    if (tid == 0) {
      sh->bin = (int)bin;
      sh->before = before;
      sh->cnt = c;
      sh->ncand = 0u;
    }
  }
  __syncthreads();
  const uint32_t bin = (uint32_t)sh->bin;
  kk -= sh->before;
  cnt = sh->cnt;
  prefix |= (uint64_t)bin << shift;
  mask |= (uint64_t)dm << shift;
  hi = shift - 1;
}

template <int NW, int VPT>
__device__ double block_select2(const uint64_t (&key)[VPT], uint32_t kth, uint64_t kmin, uint64_t kmax,
                                uint32_t* hist, uint64_t* cand, SelShared* sh) {
  const int tid = threadIdx.x;
  if (kmin == kmax) return dval(kmin);
  int hi = 63 - __builtin_clzll(kmin ^ kmax);
  uint64_t mask = (hi == 63) ? 0ull : ~((2ull << hi) - 1ull);
  uint64_t prefix = kmin & mask;
  uint32_t kk = kth, cnt = 0;
  block_select_pass<NW, VPT, kSelBits>(key, hist, sh, tid, hi, mask, prefix, kk, cnt);
  while (cnt > (uint32_t)kCandMax && hi >= 0)
    block_select_pass<NW, VPT, kSelBits2>(key, hist, sh, tid, hi, mask, prefix, kk, cnt);
  if (hi < 0) return dval(prefix);
#pragma unroll
  for (int v = 0; v < VPT; ++v)
    if ((key[v] & mask) == prefix) cand[atomicAdd(&sh->ncand, 1u)] = key[v];
  __syncthreads();
  if (tid < 64) {
    const uint64_t mine = (uint32_t)tid < cnt ? cand[tid] : ~0ull;
    uint32_t r = 0;
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint64_t o = cand[j];
      r += (o < mine) | ((o == mine) & (j < (uint32_t)tid));
    }
    const unsigned long long hit = wave_ballot((uint32_t)tid < cnt && r == kk);
    const int who = __builtin_amdgcn_readfirstlane(__ffsll((long long)hit) - 1);
    const uint64_t ans = readlane_u64(mine, who);
    if (tid == 0) sh->ans = ans;
  }
  __syncthreads();
  return dval(sh->ans);
}

template <int NW, int VPT>
__global__ __launch_bounds__(64 * NW) HB_WPE_ATTR void hb_eval_block_kernel(
    const double* __restrict__ t, const double2* __restrict__ ph, const double* __restrict__ f,
    const double* __restrict__ isg, long n,
    long kth, const WalkerConst* __restrict__ wcs, double* __restrict__ logl, double* __restrict__ tmpl_out,
    int mode) {
  constexpr int NT = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  SelShared* sh = reinterpret_cast<SelShared*>(smem);
  double* vals = reinterpret_cast<double*>(smem + sizeof(SelShared));
  uint32_t* hist = reinterpret_cast<uint32_t*>(vals);
  uint64_t* cand = reinterpret_cast<uint64_t*>(smem + sizeof(SelShared) + (4u << kSelBits));
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wv = blockIdx.x;
  const WalkerConst& w = wcs[wv];
  if (mode == 0 && w.roche != 0.0) {  // likelihood3.c:866-869, see hb_eval_kernel
    if (tid == 0) logl[wv] = -kBig / 2.0;
    return;
  }
  const int nn = (int)n;
  uint64_t kmn, kmx;
  model_pass<NT>(t, ph, nn, w, vals, tid, kmn, kmx);
  kmn = wave_reduce_u64(kmn, OpMinU64());
  kmx = wave_reduce_u64(kmx, OpMaxU64());
  if (lane == 0) {
    sh->red_min[wave] = kmn;
    sh->red_max[wave] = kmx;
  }
  __syncthreads();
  kmn = sh->red_min[0];
  kmx = sh->red_max[0];
#pragma unroll
  for (int k = 1; k < NW; ++k) {
    kmn = sh->red_min[k] < kmn ? sh->red_min[k] : kmn;
    kmx = sh->red_max[k] > kmx ? sh->red_max[k] : kmx;
  }
  // key slots v < nlive hold cadences v*NT + tid (a compare with a constant per
  // slot: no per-slot predicate is held across the select)
  const int nlive = (nn - tid + NT - 1) / NT;
  uint64_t key[VPT];
#pragma unroll
  for (int v = 0; v < VPT; ++v) key[v] = v < nlive ? dkey(vals[v * NT + tid]) : ~0ull;  // padding sorts last
  __syncthreads();  // the slab becomes the histogram
#if HB_ABLATE_SELECT
  const double med = dval(kmn);
#else
  const double med = block_select2<NW, VPT>(key, (uint32_t)kth, kmn, kmx, hist, cand, sh);
#endif
  const double blend = w.blend, one_m_blend = 1.0 - w.blend, tune = w.tune;
  if (mode == 1) {
    double* o = tmpl_out + (size_t)wv * (size_t)n;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      if (v < nlive) {
        const double m = (dval(key[v]) - med) + 1.0;
        o[v * NT + tid] = (blend + m * one_m_blend) * tune;
      }
    }
    return;
  }
  double acc = 0.0;
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const int i = v * NT + tid;
    if (v < nlive) {
      double m = (dval(key[v]) - med) + 1.0;
      m = (blend + m * one_m_blend) * tune;
      const double r = (m - f[i]) * isg[i];
      acc += r * r;
    }
  }
  acc = wave_sum_dpp(acc);
  if (lane == 0) sh->red_sum[wave] = acc;
  __syncthreads();
  if (tid == 0) {
    double chi2 = sh->red_sum[0];
#pragma unroll
    for (int k = 1; k < NW; ++k) chi2 += sh->red_sum[k];
    double c = chi2 + w.chi2_extra;
    if (w.roche != 0.0) c = kBig;
    logl[wv] = -c / 2.0;
  }
}

// ---------------------------------------------------------------------------
// auxiliary kernels for the likelihood3.h drop-in entry points
// ---------------------------------------------------------------------------
// traj(): one lane per time
__global__ void hb_traj_kernel(const double* __restrict__ times, int nt, TrajArgs ta,
                               double* __restrict__ d, double* __restrict__ z1,
                               double* __restrict__ z2, double* __restrict__ rr,
                               double* __restrict__ ff) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nt) return;
  const Orbit o = hb_orbit(times[i], ta.w);
  d[i] = o.dR;  // aR holds a in cm for this path
  rr[i] = o.rR;
  ff[i] = atan2(o.snu, o.cnu);
  const double zz = o.rR * o.su * ta.w.si;
  z1[i] = zz * ta.fz1;
  z2[i] = -zz * ta.fz2;
}

// scalar entry points, evaluated by one device lane
__global__ void hb_probe_kernel(int op, const double* __restrict__ in, double* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  switch (op) {
    case kOpAlphaBeam: out[0] = beam_coeff(in[0]); break;
    case kOpBeaming: {
      // (P, M1, M2, e, inc, omega0, nu, alpha_beam)
      const StarCoef c = star_coef(in[0], in[1], in[2], in[3], sin(in[4]), 1.0, 1.0, 0.16, 0.34, 1.0, in[7]);
      out[0] = c.kb * cos(in[5] + in[6]);
      break;
    }
    case kOpEllipsoidal: {
      // (P, M1, M2, e, inc, omega0, nu, R1, a, mu, tau)
      const double e = in[3], nu = in[6], u = in[5] + in[6];
      const StarCoef c = star_coef(in[0], in[1], in[2], e, sin(in[4]), in[7], 1.0, in[9], in[10], 1.0, 1.0);
      const double b = (1.0 + e * cos(nu)) / (1.0 - e * e);
      const double b3 = b * b * b, b4 = b3 * b, b5 = b4 * b;
      out[0] = c.am1 + b3 * (c.am2 + c.c21 * cos(2 * u)) + b4 * (c.s1 * sin(u) + c.s3 * sin(3 * u)) +
               b5 * (c.am3 + c.c22 * cos(2 * u) + c.c4 * cos(4 * u));
      break;
    }
    case kOpReflection: {
      // (P, M1, M2, e, inc, omega0, nu, R2, alpha_ref1)
      const double e = in[3], nu = in[6], u = in[5] + in[6], si = sin(in[4]);
      const StarCoef c = star_coef(in[0], in[1], in[2], e, si, 1.0, in[7], 0.16, 0.34, in[8], 1.0);
      const double b = (1.0 + e * cos(nu)) / (1.0 - e * e);
      out[0] = c.kref * (b * b) * (0.64 - si * sin(u) + 0.18 * (si * si) * (1.0 - cos(2 * u)));
      break;
    }
    case kOpEclipse: {
      double ra = in[0], rb = in[1];
      if (rb > ra) { const double k = ra; ra = rb; rb = k; }
      const double d = fabs(in[2]) / kRsun;
      out[0] = overlap_area(ra, rb, sqrt(ra * ra - rb * rb), d);
      break;
    }
    case kOpGetT: out[0] = logteff_of_mass(exp10(in[0])); break;
    case kOpGetR: out[0] = logradius_of_mass(exp10(in[0])); break;
    case kOpEnvT: out[0] = teff_spread(); break;
    case kOpEnvR: out[0] = radius_spread_of_mass(exp10(in[0])); break;
    case kOpRadiiTeffs: {
      const Stellar s = stellar_of(in);
      out[0] = s.r1; out[1] = s.r2; out[2] = s.t1; out[3] = s.t2;
      break;
    }
    case kOpMags: {
      // in[0..20] params, in[21] distance
      const Stellar s = stellar_of(in);
      const double r1 = s.r1 * kRsun, r2 = s.r2 * kRsun;
      const double mb = ab_mag(band_flux(442.0, r1, r2, s.t1, s.t2, in[21], in[19]));
      const double mv = ab_mag(band_flux(540.0, r1, r2, s.t1, s.t2, in[21], in[19]));
      const double mg = ab_mag(band_flux(673.0, r1, r2, s.t1, s.t2, in[21], in[19]));
      const double mt = ab_mag(band_flux(750.0, r1, r2, s.t1, s.t2, in[21], in[19]));
      out[0] = mg; out[1] = mb - mv; out[2] = mv - mg; out[3] = mg - mt;
      break;
    }
    case kOpRoche: {
      const double mag[5] = {1000., 1., 1., 1., 1.};
      const double err[4] = {1e15, 1e15, 1e15, 1e15};
      WalkerConst w;
      hb_prepare_walker(in, mag, err, w);
      out[0] = w.roche;
      break;
    }
    case kOpEggleton: out[0] = lobe_fraction(in[0]); break;
    default: out[0] = __builtin_nan(""); break;
  }
}

// Lomuto partition, exact reference order (likelihood3.c:48-64), one lane.
__global__ void hb_partition_kernel(double* __restrict__ a, int lo, int hi, int* __restrict__ res) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const double piv = a[hi];
  int slot = lo - 1;
  for (int k = lo; k < hi; ++k) {
    if (a[k] < piv) {
      ++slot;
      const double x = a[slot]; a[slot] = a[k]; a[k] = x;
    }
  }
  const double x = a[slot + 1]; a[slot + 1] = a[hi]; a[hi] = x;
  res[0] = slot + 1;
}

// remove_median on an array already in HBM: one 16-wave workgroup
__global__ __launch_bounds__(1024) void hb_median_kernel(double* __restrict__ a, long n, long kth) {
  __shared__ SelShared sh;
  uint64_t kmn = ~0ull, kmx = 0ull;
  for (long i = threadIdx.x; i < n; i += 1024) {
    const uint64_t k = dkey(a[i]);
    kmn = k < kmn ? k : kmn;
    kmx = k > kmx ? k : kmx;
  }
  block_minmax<16>(kmn, kmx, &sh);
  const double med = block_select<16>(a, n, kth, kmn, kmx, &sh);
  __syncthreads();
  for (long i = threadIdx.x; i < n; i += 1024) a[i] -= med;
}

// ---------------------------------------------------------------------------
// quickSort drop-in (likelihood3.c:70-83): bitonic sort of order-preserving
// 64-bit keys (dkey), padded to a power of two with ~0 (sorts last).  Up to
// kSortLds keys the whole network runs in one workgroup's LDS; beyond it the
// merge steps with a stride >= kSortLds/2 are one global launch each and the
// smaller strides of every stage finish in LDS per kSortLds-key tile.  Off the
// batched hot path (drop-in completeness); equal keys are equal values, so
// stability does not matter.
// ---------------------------------------------------------------------------
constexpr int kSortLds = 8192;  // keys per LDS tile (64 KiB)
__global__ __launch_bounds__(1024) void hb_sort_keys_kernel(const double* __restrict__ in, long n, long npad,
                                                            uint64_t* __restrict__ keys) {
  for (long i = blockIdx.x * 1024L + threadIdx.x; i < npad; i += (long)gridDim.x * 1024L)
    keys[i] = i < n ? dkey(in[i]) : ~0ull;
}
__global__ __launch_bounds__(1024) void hb_sort_vals_kernel(const uint64_t* __restrict__ keys, long n,
                                                            double* __restrict__ out) {
  for (long i = blockIdx.x * 1024L + threadIdx.x; i < n; i += (long)gridDim.x * 1024L) out[i] = dval(keys[i]);
}
__device__ __forceinline__ void cmp_swap(uint64_t& a, uint64_t& b, bool up) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = up ? lo : hi;
  b = up ? hi : lo;
}
// stages k = kfrom .. kto (doubling), strides j < min(k, tile) of each, on
// one LDS tile of `tile` keys (tile = npad when the whole sort fits); the
// direction of a pair is that of its k-block in the global index
__global__ __launch_bounds__(1024) void hb_sort_tile_kernel(uint64_t* __restrict__ keys, int tile, long kfrom,
                                                            long kto) {
  __shared__ uint64_t sk[kSortLds];
  const long base = (long)blockIdx.x * tile;
  for (int i = threadIdx.x; i < tile; i += 1024) sk[i] = keys[base + i];
  __syncthreads();
  for (long k = kfrom; k <= kto; k <<= 1) {
    for (long j = (k < tile ? k : tile) >> 1; j > 0; j >>= 1) {
      for (int q = threadIdx.x; q < tile / 2; q += 1024) {
        const int i = (int)(2 * j * (q / j) + (q % j));  // lower index of the pair
        const bool up = ((base + i) & k) == 0;
        cmp_swap(sk[i], sk[i + j], up);
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < tile; i += 1024) keys[base + i] = sk[i];
}
// one global merge step (stage k, stride j >= tile / 2)
__global__ __launch_bounds__(1024) void hb_sort_step_kernel(uint64_t* __restrict__ keys, long npad, long k,
                                                            long j) {
  for (long q = blockIdx.x * 1024L + threadIdx.x; q < npad / 2; q += (long)gridDim.x * 1024L) {
    const long i = 2 * j * (q / j) + (q % j);
    cmp_swap(keys[i], keys[i + j], (i & k) == 0);
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
hipError_t launch_prep(const double* d_params, int nwalk, const MagArgs& ma, WalkerConst* d_wc,
                       hipStream_t s, const TargetDesc* tab, const int* wt, const double* t, long n,
                       double2* ph, const int* w0, int ntargets, double* tab_pc) {
  if (nwalk <= 0) return hipSuccess;
  if (t == nullptr || (tab != nullptr && w0 == nullptr) || !HB_PHASE_TAB) ph = nullptr;
  // the most walkers per workgroup that still leave >= 256 workgroups (one per CU),
  // at most 32: both stars' lane tasks then fit one pass (prep_records); 64
  // walkers (two passes) measured 0.1648 vs 0.1640 ms per C5 call
  // (profiles/r04/r04k_c5_w*.json, interleaved)
  static const int wmax = getenv("HB_PREP_WMAX") ? atoi(getenv("HB_PREP_WMAX")) : 32;  // A/B knob
  const int nw = (wmax >= 64 && nwalk >= 256 * 64) ? 64 : (wmax >= 32 && nwalk >= 256 * 32) ? 32 : kPrepWalkers;
  const int nb = (nwalk + nw - 1) / nw;
  auto kern = nw == 64 ? hb_prep_kernel<64> : nw == 32 ? hb_prep_kernel<32> : hb_prep_kernel<kPrepWalkers>;
  hipLaunchKernelGGL(kern, dim3(nb), dim3(kPrepThreads), 0, s, d_params, nwalk, ma, d_wc, tab, wt, t,
                     (int)n, ph, w0, ntargets, tab_pc, (const int*)nullptr);
  return hipGetLastError();
}

hipError_t launch_prep_list(const double* d_params, const int* list, int count, WalkerConst* d_wc, hipStream_t s,
                            const TargetDesc* tab, const int* wt, const int* w0) {
  if (count <= 0) return hipSuccess;
  if (!list || !tab || !wt || !w0) return hipErrorInvalidValue;
  const int nw = count >= 256 * 32 ? 32 : kPrepWalkers;
  const int nb = (count + nw - 1) / nw;
  const MagArgs unused{};
  auto kern = nw == 32 ? hb_prep_kernel<32, true> : hb_prep_kernel<kPrepWalkers, true>;
  hipLaunchKernelGGL(kern, dim3(nb), dim3(kPrepThreads), 0, s, d_params, count, unused, d_wc, tab, wt,
                     (const double*)nullptr, 0, (double2*)nullptr, w0, 0, (double*)nullptr, list);
  return hipGetLastError();
}

template <int NW, int VPT>
static hipError_t launch_block_t(const EvalPlan& pl, const double* t, const double2* ph, const double* f,
                                 const double* sg,
                                 const WalkerConst* wc, int nwalk, double* logl, double* tmpl, int mode,
                                 hipStream_t s) {
  auto kern = hb_eval_block_kernel<NW, VPT>;
  static bool attr_set = false;  // per instantiation; benign race (idempotent)
  if (!attr_set && pl.lds_bytes > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds_bytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(nwalk), dim3(64 * NW), pl.lds_bytes, s, t, ph, f, sg, pl.n, pl.kth, wc, logl,
                     tmpl, mode);
  return hipGetLastError();
}

template <int NW, bool LDS>
static hipError_t launch_eval_t(const EvalPlan& pl, const double* t, const double2* ph, const double* f,
                                const double* sg,
                                const WalkerConst* wc, int nwalk, double* logl, double* tmpl,
                                double* scratch, int mode, hipStream_t s) {
  auto kern = hb_eval_kernel<NW, LDS>;
  static bool attr_set = false;  // per instantiation; benign race (idempotent)
  if (!attr_set && pl.lds_bytes > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.lds_bytes);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(nwalk), dim3(64 * NW), pl.lds_bytes, s, t, ph, f, sg, pl.n, pl.kth, wc,
                     logl, tmpl, scratch, mode);
  return hipGetLastError();
}

// Walkers per workgroup of the one-wave kernel: 16 fills a CU (4 waves per
// SIMD) with one workgroup, so the pacer (HB_PRIO == 2) sees every wave of a
// SIMD; fewer when the batch would leave CUs idle or the LDS does not fit.
#ifndef HB_WPB_MAX
#define HB_WPB_MAX 1
#endif
constexpr size_t kLdsCap = 163840;
int wave_wpb(int count, size_t lds_per) {
  int wpb = HB_WPB_MAX;
  while (wpb > 1 && ((long)count < 256L * wpb || (size_t)wpb * lds_per + 64 > kLdsCap)) wpb >>= 2;
  return wpb < 1 ? 1 : wpb;
}

template <int VPT, bool MULTI, bool ACC, int WPB, int WPW = 1, bool PRE = false>
static hipError_t launch_wave_g(size_t lds_per, int count, hipStream_t s, const double* t, const double2* ph,
                                const double* f, const double* sg, const double* rows, long n, long kth, const WalkerConst* wc,
                                double* logl, double* tmpl, int mode, size_t slab, double gap,
                                const TargetDesc* tab, const int* wt, const int* list,
                                const hbds::AccArgs& acc, double* dq, const PreArgs* pre = nullptr) {
  auto kern = hb_eval_wave_kernel<VPT, MULTI, ACC, WPB, WPW, PRE>;
  // PRE: the slices, then the LDS phase table (16 B per cadence)
  const size_t lds = (size_t)WPB * lds_per + (PRE ? (MULTI ? 0 : (((size_t)n * 16 + 15) & ~(size_t)15)) : (WPB > 1 ? 64 : 0));
  if (lds > kLdsCap) return hipErrorInvalidValue;
  static bool attr_set = false;  // per instantiation; benign race (idempotent)
  if (!attr_set && lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsCap);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((count + WPB - 1) / WPB), dim3(64 * WPB * WPW), lds, s, t, ph, f, sg, rows, n, kth, wc, logl,
                     tmpl, mode, (int)slab, gap, tab, wt, list, acc, count, (int)lds_per, dq, pre ? *pre : PreArgs{});
  return hipGetLastError();
}

// LDS bytes per walker of the fused launch: the slab, with the survivors
// inside it when it is big enough (kCandInSlab)
static size_t fused_lds_per(const EvalPlan& pl) {
  const size_t slab = pl.slab_bytes;
  return slab >= (size_t)kCandInSlab ? slab : wave_lds_bytes(slab, pl.vpt, 1);
}

// the prologue's scratch (prep records, catalog magnitudes and walker lists),
// which aliases the workgroup's slabs
static size_t fused_scratch_bytes(int wpb) {
  const size_t ps = wpb == 16 ? sizeof(PrepShared<16>) : wpb == 8 ? sizeof(PrepShared<8>) : sizeof(PrepShared<4>);
  return ps + (size_t)wpb * (3 * sizeof(double) + 2 * sizeof(int));
}

// Walkers per workgroup of the fused launch (0: prep + eval launches).  The
// workgroup keeps WPB one-wave walkers plus the LDS phase table; the largest
// WPB in {16, 8, 4} that still gives every CU a workgroup, as long as the
// resident walkers per CU (LDS) match the one-wave kernel's 16 (or the batch's
// share).  Batches beyond one resident round (w > 16 CUs) keep two launches:
// a 1024-thread workgroup frees its CU only when its slowest walker is done,
// where single-wave workgroups backfill.  HB_FUSED=0 (A/B knob): never;
// HB_FUSED=2: whenever it fits.
int fused_wpb(const EvalPlan& pl, int w, int cus) {
  static const int mode = getenv("HB_FUSED") ? atoi(getenv("HB_FUSED")) : 1;
  if (mode == 0 || pl.vpt <= 0 || pl.vpt > 16 || pl.wpw != 1 || !HB_GQ || HB_SEL_V != 3 || HB_PRIO == 2) return 0;
  if (w <= 0 || cus <= 0 || (mode == 1 && (long)w > 16L * cus)) return 0;
  const size_t per = fused_lds_per(pl), tabb = ((size_t)pl.n * 16 + 15) & ~(size_t)15;
  const long share = std::min<long>(16, ((long)w + cus - 1) / cus);  // walkers a CU must hold at once
  for (int wpb = 16; wpb >= 4; wpb >>= 1) {
    const size_t lds = (size_t)wpb * per + tabb;
    if (lds > kLdsCap || fused_scratch_bytes(wpb) > (size_t)wpb * per) continue;
    const long resident = (long)(kLdsCap / lds) * wpb;
    if (resident < share) continue;
    if (wpb > 4 && ((long)w + wpb - 1) / wpb < cus) continue;  // a workgroup for every CU
    return wpb;
  }
  return 0;
}

template <int VPT>
static hipError_t launch_fused_t(const EvalPlan& pl, int wpb, const PreArgs& pa, const double* t, const double* f,
                                 const double* sg, const double* rows, int nwalk, double* logl, hipStream_t s,
                                 double* dq) {
  const size_t per = fused_lds_per(pl);
  const hbds::AccArgs none{};
#define HB_FCASE(WV)                                                                                               \
  if (wpb == WV)                                                                                                   \
    return launch_wave_g<VPT, false, false, WV, 1, true>(per, nwalk, s, t, pa.ph, f, sg, rows, pl.n, pl.kth, pa.wc, \
                                                         logl, nullptr, 0, pl.slab_bytes, pl.gap, nullptr, nullptr,  \
                                                         nullptr, none, dq, &pa);
  HB_FCASE(16)
  HB_FCASE(8)
  HB_FCASE(4)
#undef HB_FCASE
  return hipErrorInvalidValue;
}

// catalog mode, records in the prologue: one size class of one-wave walkers.
// 16 walkers per workgroup while their slabs fit LDS (the prep roles' issue
// per walker falls with the walkers sharing a workgroup), else 8 / 4.
template <int VPT>
static hipError_t launch_multi_fused_t(size_t slab, const PreArgs& pa, const double* t, const double* f,
                                       const double* sg, const double* rows, int count, double* logl, hipStream_t s,
                                       double* dq) {
  EvalPlan pl;
  pl.vpt = VPT;
  pl.slab_bytes = slab;
  const size_t per = fused_lds_per(pl);
  const hbds::AccArgs none{};
#define HB_MFCASE(WV)                                                                                            \
  if ((size_t)WV * per <= kLdsCap && fused_scratch_bytes(WV) <= (size_t)WV * per)                                \
    return launch_wave_g<VPT, true, false, WV, 1, true>(per, count, s, t, nullptr, f, sg, rows, 0L, 0L, pa.wc,   \
                                                        logl, nullptr, 0, slab, 0.0, pa.tab, pa.wt, pa.list, none, \
                                                        dq, &pa);
  if (count >= 64) {
    HB_MFCASE(16)
  }
  if (count >= 16) {
    HB_MFCASE(8)
  }
  HB_MFCASE(4)
#undef HB_MFCASE
  return hipErrorInvalidValue;
}

hipError_t launch_eval_multi_fused(int vpt, size_t slab, const PreArgs& pa, const double* t, const double* f,
                                   const double* sg, const double* rows, int count, double* logl, hipStream_t s,
                                   double* dq) {
  if (count <= 0) return hipSuccess;
  if (!HB_PIPE || !HB_CHAIN_SPLIT || dq == nullptr || pa.params == nullptr || pa.wc == nullptr || pa.list == nullptr ||
      pa.wt == nullptr || pa.tab == nullptr || pa.w0 == nullptr)
    return hipErrorInvalidValue;
  switch (vpt) {
    case 1: return launch_multi_fused_t<1>(slab, pa, t, f, sg, rows, count, logl, s, dq);
    case 2: return launch_multi_fused_t<2>(slab, pa, t, f, sg, rows, count, logl, s, dq);
    case 4: return launch_multi_fused_t<4>(slab, pa, t, f, sg, rows, count, logl, s, dq);
    case 8: return launch_multi_fused_t<8>(slab, pa, t, f, sg, rows, count, logl, s, dq);
    case 16: return launch_multi_fused_t<16>(slab, pa, t, f, sg, rows, count, logl, s, dq);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_eval_fused(const EvalPlan& pl, int wpb, const PreArgs& pa, const double* t, const double* f,
                             const double* sg, const double* rows, int nwalk, double* logl, hipStream_t s, double* dq) {
  if (nwalk <= 0) return hipSuccess;
  if (dq == nullptr || pa.params == nullptr || pa.wc == nullptr || pa.ph == nullptr) return hipErrorInvalidValue;
  switch (pl.vpt) {
    case 1: return launch_fused_t<1>(pl, wpb, pa, t, f, sg, rows, nwalk, logl, s, dq);
    case 2: return launch_fused_t<2>(pl, wpb, pa, t, f, sg, rows, nwalk, logl, s, dq);
    case 4: return launch_fused_t<4>(pl, wpb, pa, t, f, sg, rows, nwalk, logl, s, dq);
    case 8: return launch_fused_t<8>(pl, wpb, pa, t, f, sg, rows, nwalk, logl, s, dq);
    case 16: return launch_fused_t<16>(pl, wpb, pa, t, f, sg, rows, nwalk, logl, s, dq);
    default: return hipErrorInvalidValue;
  }
}

template <int VPT, bool MULTI, bool ACC, int WPW = 1>
static hipError_t launch_wave_w(size_t slab, int count, hipStream_t s, const double* t, const double2* ph,
                                const double* f, const double* sg, const double* rows, long n, long kth, const WalkerConst* wc,
                                double* logl, double* tmpl, int mode, double gap, const TargetDesc* tab,
                                const int* wt, const int* list, const hbds::AccArgs& acc, double* dq) {
  const size_t per = wave_lds_bytes(slab, VPT, WPW);
  if constexpr (WPW > 1)  // a pair of waves per walker: one walker per workgroup
    return launch_wave_g<VPT, MULTI, ACC, 1, WPW>(per, count, s, t, ph, f, sg, rows, n, kth, wc, logl, tmpl, mode,
                                                  slab, gap, tab, wt, list, acc, dq);
  switch (wave_wpb(count, per)) {
#if HB_WPB_MAX >= 16
    case 16:
      return launch_wave_g<VPT, MULTI, ACC, 16>(per, count, s, t, ph, f, sg, rows, n, kth, wc, logl, tmpl, mode, slab,
                                                gap, tab, wt, list, acc, dq);
#endif
#if HB_WPB_MAX >= 4
    case 4:
      return launch_wave_g<VPT, MULTI, ACC, 4>(per, count, s, t, ph, f, sg, rows, n, kth, wc, logl, tmpl, mode, slab,
                                               gap, tab, wt, list, acc, dq);
#endif
    default:
      return launch_wave_g<VPT, MULTI, ACC, 1>(per, count, s, t, ph, f, sg, rows, n, kth, wc, logl, tmpl, mode, slab,
                                               gap, tab, wt, list, acc, dq);
  }
}

template <int VPT>
static hipError_t launch_wave_t(const EvalPlan& pl, const double* t, const double2* ph, const double* f,
                                const double* sg, const double* rows,
                                const WalkerConst* wc, int nwalk, double* logl, double* tmpl, int mode,
                                hipStream_t s, double* dq) {
#define HB_WPW_CASE(WV)                                                                                      \
  if (pl.wpw == WV)                                                                                          \
    return launch_wave_w<VPT, false, false, WV>(pl.slab_bytes, nwalk, s, t, ph, f, sg, rows, pl.n, pl.kth, wc, logl, \
                                                tmpl, mode, pl.gap, nullptr, nullptr, nullptr, hbds::AccArgs{}, dq);
  if constexpr (VPT == 16 || VPT == 8) {
    HB_WPW_CASE(2)
  }
  if constexpr (VPT == 16) {
    HB_WPW_CASE(4)
    HB_WPW_CASE(8)
    HB_WPW_CASE(16)
  }
  if constexpr (VPT == 32) {
    HB_WPW_CASE(16)
  }
#undef HB_WPW_CASE
  if (pl.wpw != 1) return hipErrorInvalidValue;
  return launch_wave_w<VPT, false, false>(pl.slab_bytes, nwalk, s, t, ph, f, sg, rows, pl.n, pl.kth, wc, logl, tmpl,
                                          mode, pl.gap, nullptr, nullptr, nullptr, hbds::AccArgs{}, dq);
}

template <int VPT>
static hipError_t launch_wave_acc_t(const EvalPlan& pl, const double* t, const double2* ph, const double* f,
                                    const double* sg, const double* rows, const WalkerConst* wc, int nwalk,
                                    double* logl, hipStream_t s, const hbds::AccArgs& acc, double* dq) {
  return launch_wave_w<VPT, false, true>(pl.slab_bytes, nwalk, s, t, ph, f, sg, rows, pl.n, pl.kth, wc, logl, nullptr,
                                         0, pl.gap, nullptr, nullptr, nullptr, acc, dq);
}

template <int VPT>
static hipError_t launch_multi_t(size_t slab, const double* t, const double2* ph, const double* f,
                                 const double* sg, const double* rows,
                                 const TargetDesc* tab, const int* wt, const int* list, int count,
                                 const WalkerConst* wc, double* logl, hipStream_t s, double* dq, int wpw) {
  if constexpr (VPT == 16 || VPT == 8)
    if (wpw == 2)
      return launch_wave_w<VPT, true, false, 2>(slab, count, s, t, ph, f, sg, rows, 0L, 0L, wc, logl, nullptr, 0, 0.0,
                                                tab, wt, list, hbds::AccArgs{}, dq);
  if (wpw != 1) return hipErrorInvalidValue;
  return launch_wave_w<VPT, true, false>(slab, count, s, t, ph, f, sg, rows, 0L, 0L, wc, logl, nullptr, 0, 0.0, tab, wt,
                                         list, hbds::AccArgs{}, dq);
}

hipError_t launch_eval_multi(int vpt, size_t slab, const double* t, const double2* ph, const double* f,
                             const double* sg, const double* rows,
                             const TargetDesc* tab, const int* wt, const int* list, int count,
                             const WalkerConst* wc, double* logl, hipStream_t s, double* dq, int wpw) {
  if (count <= 0) return hipSuccess;
  switch (vpt) {
    case 1: return launch_multi_t<1>(slab, t, ph, f, sg, rows, tab, wt, list, count, wc, logl, s, dq, wpw);
    case 2: return launch_multi_t<2>(slab, t, ph, f, sg, rows, tab, wt, list, count, wc, logl, s, dq, wpw);
    case 4: return launch_multi_t<4>(slab, t, ph, f, sg, rows, tab, wt, list, count, wc, logl, s, dq, wpw);
    case 8: return launch_multi_t<8>(slab, t, ph, f, sg, rows, tab, wt, list, count, wc, logl, s, dq, wpw);
    case 16: return launch_multi_t<16>(slab, t, ph, f, sg, rows, tab, wt, list, count, wc, logl, s, dq, wpw);
    case 32: return launch_multi_t<32>(slab, t, ph, f, sg, rows, tab, wt, list, count, wc, logl, s, dq, wpw);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_eval(const EvalPlan& pl, const double* t, const double2* ph, const double* f, const double* sg,
                       const double* rows, const WalkerConst* wc, int nwalk, double* logl, double* tmpl, double* scratch,
                       int mode, hipStream_t s, const hbds::AccArgs* acc, double* dq) {
  if (nwalk <= 0) return hipSuccess;
  if (pl.vpt > 0 && HB_GQ && dq == nullptr) return hipErrorInvalidValue;  // the one-wave path's deferred queue
  if (acc != nullptr) {  // fused Hastings epilogue: one-wave path only
    if (mode != 0) return hipErrorInvalidValue;
    if (pl.wpw != 1) return hipErrorNotSupported;
    switch (pl.vpt) {
      case 1: return launch_wave_acc_t<1>(pl, t, ph, f, sg, rows, wc, nwalk, logl, s, *acc, dq);
      case 2: return launch_wave_acc_t<2>(pl, t, ph, f, sg, rows, wc, nwalk, logl, s, *acc, dq);
      case 4: return launch_wave_acc_t<4>(pl, t, ph, f, sg, rows, wc, nwalk, logl, s, *acc, dq);
      case 8: return launch_wave_acc_t<8>(pl, t, ph, f, sg, rows, wc, nwalk, logl, s, *acc, dq);
      case 16: return launch_wave_acc_t<16>(pl, t, ph, f, sg, rows, wc, nwalk, logl, s, *acc, dq);
      // 32 cadences per lane: the epilogue's registers would spill (22 VGPRs):
      // the device sampler launches ds_accept (hbx_loglik_accept_dev returns 1)
      default: return hipErrorNotSupported;
    }
  }
  switch (pl.vpt) {
    case 0: break;
    case 1: return launch_wave_t<1>(pl, t, ph, f, sg, rows, wc, nwalk, logl, tmpl, mode, s, dq);
    case 2: return launch_wave_t<2>(pl, t, ph, f, sg, rows, wc, nwalk, logl, tmpl, mode, s, dq);
    case 4: return launch_wave_t<4>(pl, t, ph, f, sg, rows, wc, nwalk, logl, tmpl, mode, s, dq);
    case 8: return launch_wave_t<8>(pl, t, ph, f, sg, rows, wc, nwalk, logl, tmpl, mode, s, dq);
    case 16: return launch_wave_t<16>(pl, t, ph, f, sg, rows, wc, nwalk, logl, tmpl, mode, s, dq);
    case 32: return launch_wave_t<32>(pl, t, ph, f, sg, rows, wc, nwalk, logl, tmpl, mode, s, dq);
    default: return hipErrorInvalidValue;
  }
  if (pl.bvpt > 0) {
#define HB_BCASE(NWV, V)                                                                    \
  if (pl.nw == NWV && pl.bvpt == V) return launch_block_t<NWV, V>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, mode, s);
    HB_BCASE(4, 8) HB_BCASE(4, 16) HB_BCASE(4, 20)
    HB_BCASE(8, 8) HB_BCASE(8, 16) HB_BCASE(8, 20)
    HB_BCASE(16, 8) HB_BCASE(16, 16) HB_BCASE(16, 20)
#undef HB_BCASE
    return hipErrorInvalidValue;
  }
  // the template in LDS always takes the register-key block kernel above
  // (HB_BLOCK_KEYS); the LDS-walking select is built only without it
#if HB_BLOCK_KEYS
#define HB_CASE(NWV)                                                                              \
  case NWV:                                                                                       \
    return pl.lds ? hipErrorInvalidValue                                                          \
                  : launch_eval_t<NWV, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
#else
#define HB_CASE(NWV)                                                                              \
  case NWV:                                                                                       \
    return pl.lds ? launch_eval_t<NWV, true>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s) \
                  : launch_eval_t<NWV, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
#endif
  switch (pl.nw) {
    HB_CASE(1)
    HB_CASE(2)
    HB_CASE(4)
    HB_CASE(8)
    HB_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef HB_CASE
}

hipError_t launch_traj(const double* d_times, int nt, const TrajArgs& ta, double* d, double* z1,
                       double* z2, double* rr, double* ff, hipStream_t s) {
  if (nt <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb_traj_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, d_times, nt, ta, d, z1, z2,
                     rr, ff);
  return hipGetLastError();
}

hipError_t launch_probe(int op, const double* d_in, double* d_out, hipStream_t s) {
  hipLaunchKernelGGL(hb_probe_kernel, dim3(1), dim3(64), 0, s, op, d_in, d_out);
  return hipGetLastError();
}

hipError_t launch_partition(double* d_a, int lo, int hi, int* d_res, hipStream_t s) {
  hipLaunchKernelGGL(hb_partition_kernel, dim3(1), dim3(64), 0, s, d_a, lo, hi, d_res);
  return hipGetLastError();
}

hipError_t launch_sort(const double* d_in, double* d_out, uint64_t* d_keys, long n, hipStream_t s) {
  if (n <= 1) {
    if (n == 1) return hipMemcpyAsync(d_out, d_in, 8, hipMemcpyDeviceToDevice, s);
    return hipSuccess;
  }
  long npad = 1;
  while (npad < n) npad <<= 1;
  const int grid = (int)std::min<long>((npad + 1023) / 1024, 4096);
  hipLaunchKernelGGL(hb_sort_keys_kernel, dim3(grid), dim3(1024), 0, s, d_in, n, npad, d_keys);
  const int tile = (int)std::min<long>(npad, kSortLds);
  const int ntile = (int)(npad / tile);
  // stages up to the tile size entirely in LDS
  hipLaunchKernelGGL(hb_sort_tile_kernel, dim3(ntile), dim3(1024), 0, s, d_keys, tile, 2L, (long)tile);
  for (long k = 2L * tile; k <= npad; k <<= 1) {
    for (long j = k >> 1; j >= tile; j >>= 1)
      hipLaunchKernelGGL(hb_sort_step_kernel, dim3(grid), dim3(1024), 0, s, d_keys, npad, k, j);
    hipLaunchKernelGGL(hb_sort_tile_kernel, dim3(ntile), dim3(1024), 0, s, d_keys, tile, k, k);
  }
  hipLaunchKernelGGL(hb_sort_vals_kernel, dim3(grid), dim3(1024), 0, s, d_keys, n, d_out);
  return hipGetLastError();
}

hipError_t launch_median(double* d_a, long n, long kth, hipStream_t s) {
  hipLaunchKernelGGL(hb_median_kernel, dim3(1), dim3(1024), 0, s, d_a, n, kth);
  return hipGetLastError();
}

// Choose waves-per-walker and template storage for N cadences.
hipError_t preload_code_object() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&hb_prep_kernel<kPrepWalkers>));
}

// lane rows per walker: 128 (a pair of waves, WPW = 2) for 1280 < n <= 2048,
// else 64.  At 4096 walkers the pair takes N = 1500 / 1861 / 2048 in 64 / 72 /
// 73 us instead of 72 / 88 / 88, and loses at N = 1100 (61 vs 55 us: chains
// of 5 cadences per lane), so short rows stay one wave.  HB_NO_PAIR=1 (A/B
// knob): one wave of 32 cadences per lane up to 2048.
#ifndef HB_PAIR_NMIN
#define HB_PAIR_NMIN (64 * 20 + 1)  // experiment knob: smallest N of the pair plan
#endif
constexpr long kPairNmin = HB_PAIR_NMIN;
//
// Above 2048 cadences the same code runs with WPW = 4 waves of lane rows per
// walker (the rows kernel: 256 rows of <= 16 cadences, warm Kepler chains)
// up to N = 4096, where it beats the block kernel (4096 walkers, HIP events:
// N = 3000 127 vs 130 us, N = 4001 145 vs 159); above, the block kernel is
// faster (8192: 329 vs 305; 20 000 with 16 waves of rows: 1179 vs 890 --
// the rows' deferred eclipse queue goes through HBM, the block kernel's
// eclipse terms stay in LDS), so 0 = no rows plan there.  (8 / 16 waves of
// rows remain instantiable for experiments.)  HB_NO_ROWS=1 (A/B knob): the
// block kernel above 2048.
constexpr long kRowsNmax = 64 * 4 * 16;
int wave_nr_for(long n) {
  static const bool no_pair = getenv("HB_NO_PAIR") != nullptr && atoi(getenv("HB_NO_PAIR")) != 0;
  static const bool no_rows = getenv("HB_NO_ROWS") != nullptr && atoi(getenv("HB_NO_ROWS")) != 0;
  if (n <= 64 * 32) return (n >= kPairNmin && !no_pair) ? 128 : 64;
  if (no_rows || n > kRowsNmax) return 0;
  return 256;
}

// cadences per lane (a power of two) of the one-wave path, 0 if n > 2048
int wave_vpt_for(long n) {
  const long nr = wave_nr_for(n);
  if (nr == 0) return 0;
  int vpt = 1;
  while ((long)vpt * nr < n) vpt <<= 1;
  return vpt;
}

// the template slab (nr lane rows of VPT doubles) doubles as the
// 2^kSelBits-bin histogram of the select
size_t wave_slab_bytes(long n) {
  const long nr = wave_nr_for(n);
  const int rc = (int)((n + nr - 1) / nr);
  const long live = (n + rc - 1) / rc;
  int stride = rows_stride(rc);
  if (nr > 128 && live * stride * 8 > kRowsLdsCap) stride = rc;  // as make_rows
  const size_t vals = (size_t)(nr > 128 ? live : nr) * stride * 8;
  const size_t slab = vals > (size_t)(4u << kSelBits) ? vals : (size_t)(4u << kSelBits);
  return (slab + 15) & ~(size_t)15;
}

// bytes of the one-wave kernel's deferred queue for `count` walkers of wpw
// waves (HB_GQ)
size_t wave_queue_bytes(int vpt, long count, int wpw) {
  return HB_GQ ? (size_t)count * (size_t)wpw * ((size_t)64 * (size_t)vpt + kDqSink) * 16 : 0;
}

// slab | select candidates | eclipse queue (chain model pass only) | the
// pair's shared words (wpw = 2)
size_t wave_lds_bytes(size_t slab, int vpt, int wpw) {
  const bool chain = vpt >= HB_CHAIN_VPT_MIN && vpt <= HB_CHAIN_VPT_MAX;
  const size_t q = (chain && !HB_GQ) ? (size_t)(kEclQ + 1) * (8 + 4) : 0;  // eclipse queue aliases the candidates
  const size_t cb = 8 * (size_t)kCandMax;
  return (slab + (q > cb ? q : cb) + (wpw > 1 ? sizeof(PairShared) : 0) + 15) & ~(size_t)15;
}

// t, f and 1/sigma in the one-wave kernel's lane-row order: row block c holds
// cadence l * rc + c for lane rows l = 0..nr-1 (nr = wave_nr_for(n), rc =
// ceil(n / nr); cadences past the end repeat the last one and are never used)
long wave_rows_doubles(long n) {
  const long nr = wave_nr_for(n);
  return 3L * nr * ((n + nr - 1) / nr);
}
void build_rows(const double* t, const double* f, const double* isg, long n, double* out) {
  const long nr = wave_nr_for(n);
  const long rc = (n + nr - 1) / nr;
  for (long c = 0; c < rc; ++c)
    for (long l = 0; l < nr; ++l) {
      const long i = std::min(l * rc + c, n - 1);
      out[c * nr + l] = t[i];
      out[nr * rc + c * nr + l] = f[i];
      out[2 * nr * rc + c * nr + l] = isg[i];
    }
}

double cadence_gap(const double* t, long n) {
  if (n < 2) return 0.0;
  std::vector<double> g((size_t)(n - 1));
  for (long i = 0; i + 1 < n; ++i) g[(size_t)i] = fabs(t[i + 1] - t[i]);
  const size_t q = (size_t)((n - 1) * 9 / 10);
  std::nth_element(g.begin(), g.begin() + q, g.end());
  const double v = g[q];
  return v == v ? v : __builtin_inf();  // NaN spacing: never warm
}

EvalPlan make_plan(long n) {
  EvalPlan pl;
  pl.n = n;
  pl.kth = (n % 2 == 0) ? n / 2 : n / 2 + 1;  // likelihood3.c:97-99
  static const long wave_max = getenv("HB_WAVE_NMAX") ? atol(getenv("HB_WAVE_NMAX")) : 64 * 32;  // A/B knob
  if ((n <= wave_max || n > 64 * 32) && wave_nr_for(n) > 0) {  // one wave (or 2..16) per walker, keys in registers
    pl.vpt = wave_vpt_for(n);
    pl.wpw = wave_nr_for(n) / 64;
    pl.nw = pl.wpw;  // waves per walker (hb_ctx_waves_per_walker)
    pl.lds = true;
    pl.slab_bytes = wave_slab_bytes(n);
    pl.lds_bytes = wave_lds_bytes(pl.slab_bytes, pl.vpt, pl.wpw);
    return pl;
  }
  return make_block_plan(n);
}

// NW waves per walker (N > 2048; for N <= 2048 the latency plan of small
// batches, hb_capi.hip run_batch): the walker's cadences over more SIMDs
EvalPlan make_block_plan(long n) {
  EvalPlan pl;
  pl.n = n;
  pl.kth = (n % 2 == 0) ? n / 2 : n / 2 + 1;  // likelihood3.c:97-99
  const size_t lds_cap = 163840;
  const size_t need = sizeof(SelShared) + (size_t)n * sizeof(double);
  if (need <= lds_cap) {
    pl.lds = true;
    pl.lds_bytes = need;
    const size_t blocks_per_cu = lds_cap / need;  // LDS-limited residency
    int nw = 1;
    while (nw < 16 && (size_t)nw * blocks_per_cu < 16) nw <<= 1;
    if (nw < 4) nw = 4;
    pl.nw = nw;
#if HB_BLOCK_KEYS
    const long per = (n + 64L * nw - 1) / (64L * nw);  // cadences per thread
    if (per <= 32 && need >= sizeof(SelShared) + (4u << kSelBits) + 8 * kCandMax)
      // exact fit at 17..20 (C3: N = 20 000 over 16 waves is 19.5 per thread): 24
      // key slots there cost <16, 24> 14 VGPR spills (64 B of scratch per lane).
      // Whenever the slab fits LDS, per <= 20 (N <= 20 300 over 16 waves; fewer
      // waves only for shorter light curves), so 24 / 32 keys are never needed
      // (and not instantiated: they spill)
      pl.bvpt = per <= 8 ? 8 : per <= 16 ? 16 : per <= 20 ? 20 : 0;
#endif
  } else {
    pl.lds = false;
    pl.lds_bytes = sizeof(SelShared);
    pl.nw = 4;
  }
  return pl;
}

}  // namespace hbk

#ifdef HB_CHAIN_STATS
extern "C" int hb_dbg_chain_stats(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hbdev::hb_chain_stats), 8 * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    unsigned long long z[8] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(hbdev::hb_chain_stats), z, sizeof z);
  }
  return e == hipSuccess ? 0 : -1;
}
#endif

#ifdef HB_WAVE_CLOCKS
extern "C" int hb_debug_prologue_clocks(unsigned long long* out, int nwg) {
  if (nwg > 4096) nwg = 4096;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hb_pro_clk), 16 * sizeof(unsigned long long) * nwg);
  return e == hipSuccess ? 0 : -1;
}
extern "C" int hb_debug_wave_clocks(unsigned long long* out, int nwaves) {
  if (nwaves > 65536) nwaves = 65536;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hb_wave_clk), 8 * sizeof(unsigned long long) * nwaves);
  return e == hipSuccess ? 0 : -1;
}
#endif
