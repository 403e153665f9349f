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
#include <stddef.h>
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

// the one-wave kernels at <= 128 VGPRs: 4 waves per SIMD (C2's 4096 walkers
// are one resident round of 16 per CU)
#define HB_WPE_ATTR __attribute__((amdgpu_waves_per_eu(4)))
// Experiment builds only (HB_WAVE_CLOCKS): per-wave shader clock at entry and
// exit plus HW_ID / XCC_ID, read back by hb_debug_wave_clocks().
#ifdef HB_WAVE_CLOCKS
// 10 words per wave: start, phase marks 0..2 (after the model pass, the keys,
// the select; 0 if not reached), end, HW_ID, XCC_ID, mark 3 (the model loop's
// end, before the deferred queue is applied), s_memrealtime (100 MHz) at start
// and end: the in-kernel shader clock is d memtime / d memrealtime x 100 MHz
// (MI355X_MICROARCH.md, DVFS give-back item 6)
constexpr int kClkWords = 10;
__device__ unsigned long long hb_wave_clk[kClkWords * 65536];
#define HB_CLK_BEGIN()                                                 \
  const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();    \
  const unsigned long long clk0_ = __builtin_amdgcn_s_memtime();       \
  unsigned long long clkm_[4] = {0ull, 0ull, 0ull, 0ull}
#define HB_CLK_MARK(i) clkm_[(i)] = __builtin_amdgcn_s_memtime()
#define HB_CLK_END(wv)                                                                          \
  do {                                                                                          \
    const unsigned long long clk1_ = __builtin_amdgcn_s_memtime();                              \
    const unsigned long long rt1_ = __builtin_amdgcn_s_memrealtime();                           \
    if ((threadIdx.x & 63) == 0 && (wv) < 65536) {                                              \
      unsigned long long* o_ = hb_wave_clk + kClkWords * (wv);                                  \
      o_[0] = clk0_;                                                                            \
      o_[1] = clkm_[0];                                                                         \
      o_[2] = clkm_[1];                                                                         \
      o_[3] = clkm_[2];                                                                         \
      o_[4] = clk1_;                                                                            \
      o_[5] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                              \
      o_[6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);                             \
      o_[7] = clkm_[3];                                                                         \
      o_[8] = rt0_;                                                                             \
      o_[9] = rt1_;                                                                             \
    }                                                                                           \
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
#endif
#include "hb_wave.hpp"

namespace hbk {

// ---------------------------------------------------------------------------
// kernel 1: per-walker constants (hb_prep.hpp), kPrepWalkers walkers per
// 256-thread workgroup (a prep group: four role waves, lane = walker), so
// W = 4096 launches 256 workgroups, one per CU.  Parameters and records move
// through LDS so the HBM accesses coalesce.  The device sampler computes the
// same records in ds_propose's epilogue instead (no launch per iteration).
// ---------------------------------------------------------------------------
constexpr int kPrepWalkers = 16;  // walkers per prep workgroup (small batches)
constexpr int kPrepThreads = 64 * kPrepRoles;

// NW walkers per workgroup: kPrepWalkers, or 32 / 64 for batches that still
// fill 256 workgroups with them (C4, C5: one round instead of two or four)
template <int NW>
__global__ __launch_bounds__(kPrepThreads) void hb_prep_kernel(const double* __restrict__ params,
                                                              int nwalk, MagArgs ma,
                                                              WalkerConst* __restrict__ out,
                                                              const TargetDesc* __restrict__ tab,
                                                              const int* __restrict__ wt,
                                                              const double* __restrict__ tcad, int ncad,
                                                              double2* __restrict__ ph,
                                                              const int* __restrict__ cw0,
                                                              const int* __restrict__ wf,
                                                              double* __restrict__ tab_pc_out) {
  constexpr int kPrepWalkers = NW;
  __shared__ PrepShared<kPrepWalkers> L;
  HB_PCLK(0, 0);  // clock builds: 0 entry, 1 parameters in LDS, 2 records stored, 3/4 waves 0/3 done
  const int G = (int)gridDim.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int base = blockIdx.x * kPrepWalkers;
  const int nb = min(kPrepWalkers, nwalk - base);
  // wave 2 writes a single context's shared-period phase table in its slack;
  // its first operands are in flight with the parameters
  const bool tabwave = ph != nullptr && tab == nullptr && (tid >> 6) == 2;
  double t_first = 0.0, lp0 = 0.0;
  if (tabwave) {
    const int i0 = blockIdx.x + G * lane;
    if (i0 < ncad) t_first = tcad[i0];
    lp0 = params[2];
  }
  // catalog phase tables: cadence ic of the concatenated arrays (grid-wide,
  // one or two per thread), its time and its target's first walker in flight now
  const bool cattab = ph != nullptr && tab != nullptr;
  const int ic = blockIdx.x * kPrepThreads + tid;
  int cw_first = -1;
  double tc_first = 0.0;
  if (cattab && ic < ncad) {
    cw_first = cw0[ic];
    tc_first = tcad[ic];
  }
  {  // all loads in flight before the first LDS write (a rolled loop serialises on vmcnt(0))
    constexpr int U = (kPrepWalkers * kNpars + kPrepThreads - 1) / kPrepThreads;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kPrepThreads;
      v[u] = i < nb * kNpars ? params[(size_t)base * kNpars + i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * kPrepThreads;
      if (i < nb * kNpars) L.sp[i] = v[u];
    }
  }
  __syncthreads();
  HB_PCLK(1, 0);
  const double lpc_first = cw_first >= 0 ? params[(size_t)cw_first * kNpars + 2] : 0.0;
  // the table period: walker 0's (single context) or the first walker's of
  // the walker's target in this batch (catalog)
  auto tab_pc = [&](int j) -> double {
    if (ph == nullptr) return __builtin_nan("");
    return exp10(params[(tab ? (size_t)wf[base + j] * kNpars : 0) + 2]) * kDay;
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
      if (i < nb * kWcDoubles) dst[i] = v[u];
    }
  }
  HB_PCLK(2, 0);
  // Catalog phase tables (WalkerConst::tab), written after the walker records
  // so their latency overlaps the stores: cadence i of target k, for the
  // period of k's first walker cw0[i] in this batch (-1: no walkers), ph[i] =
  // (sin, cos)(t_i DAY 2pi/Pc0).  Spread over the whole grid, operands loaded
  // at entry: one per thread at C5 (a target per workgroup, up to 8 cadences
  // per thread in turn, measured 12.2 us per records launch).  (A single
  // context's table is written by wave 2 above.)
  if (cattab) {
    const int gs = G * kPrepThreads;
    for (int i = ic; i < ncad; i += gs) {
      const bool fst = i == ic;
      const int cw = fst ? cw_first : cw0[i];
      if (cw < 0) continue;
      const double mA0 = kTwoPi / (exp10(fst ? lpc_first : params[(size_t)cw * kNpars + 2]) * kDay);
      double sv, cv;
      sincos_table(((fst ? tc_first : tcad[i]) * kDay) * mA0, sv, cv);
      ph[i] = make_double2(sv, cv);
    }
  }
  HB_PCLK(3, 0);
  HB_PCLK(4, 192);
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

// Model flux for cadences tid, tid+NT, ... : kK interleaved cadences per lane
// per iteration (ILP for the fp64 Kepler chains), next iteration's times
// prefetched; values go to vals[], min/max order keys returned per lane.
#ifndef HB_BLK_K
#define HB_BLK_K kK  // A/B knob: cadences interleaved per thread in the block kernels' model pass
#endif
template <int NT>
__device__ __forceinline__ void model_pass(const double* __restrict__ t, const double2* __restrict__ ph, int n,
                                           const WalkerConst& w, double* vals, int tid, uint64_t& kmn_out,
                                           uint64_t& kmx_out) {
  constexpr int K = HB_BLK_K;
  const bool tab = (ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  // running min/max as doubles (v_min/v_max_f64); NaN lanes are tracked and
  // the order keys recomputed from vals[] in that (never observed) case
  double vmn = __builtin_inf(), vmx = -__builtin_inf();
  bool nan = false;
  const int last = n - 1;
  double tk[K];
  double2 pk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = min(k * NT + tid, last);
    tk[k] = t[i];
    pk[k] = tab ? ph[i] : make_double2(0.0, 1.0);
  }
  for (int base = 0; base < n; base += K * NT) {
    double tn[K];
    double2 pn[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = min(base + (K + k) * NT + tid, last);
      tn[k] = t[i];
      pn[k] = tab ? ph[i] : make_double2(0.0, 1.0);
    }
    double v[K];
    bool bad;
    __asm__ volatile("" ::: "memory");  // walker constants reloaded per tile (see hb_cadence_flux_k)
    hb_cadence_flux_k<K>(tk, pk, tab, w, v, bad);
    if (wave_any(bad)) {  // out-of-domain angles: reference-order ocml path
      if (bad) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = hb_cadence_flux_slow(tk[k], &w);
      }
    }
    if (base + K * NT <= n) {  // full tile: no per-cadence bounds test
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
  // Roche overflow, |e| > 1: the logL needs no light curve (block-uniform
  // exit, logl_without_light_curve)
  double ll0;
  if (mode == 0 && logl_without_light_curve(w, ll0)) {
    if (tid == 0) logl[wv] = ll0;
    return;
  }

  // 1. model flux for every cadence
  uint64_t kmn, kmx;
  model_pass<NT>(t, ph, (int)n, w, vals, tid, kmn, kmx);
  __syncthreads();
  block_minmax<NW>(kmn, kmx, sh);

  // 2. median (element of rank kth in ascending order)
  const double med = block_select<NW>(vals, n, kth, kmn, kmx, sh);

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
template <int WPB>
__device__ __forceinline__ void fused_prologue(const PreArgs& pa, int count, int n, const double* __restrict__ t,
                                               unsigned char* smem_all, double2* tabl) {
  static_assert(WPB >= kPrepRoles && WPB <= 16, "four prep roles, <= 1024 threads");
  constexpr int NT = 64 * WPB;
  PrepShared<WPB>& L = *reinterpret_cast<PrepShared<WPB>*>(smem_all);
  const int tid = threadIdx.x;
  HB_PCLK(0, 0);
  const int base = blockIdx.x * WPB;
  const int nb = min(WPB, count - base);
  {  // parameters, all loads in flight before the first LDS write
    constexpr int U = (WPB * kNpars + NT - 1) / NT;
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      v[u] = i < nb * kNpars ? pa.params[(size_t)base * kNpars + i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      if (i < nb * kNpars) L.sp[i] = v[u];
    }
  }
  // the table period: walker 0's (hb_prep_kernel's tab_pc of a single context)
  const double Pc0 = exp10(pa.params[2]) * kDay;
  auto tab_pc = [&](int) -> double { return Pc0; };
  // The previous fused launch left the global table complete for Pc0 (the
  // sampler's and the bench's steady state: the period is a sampler
  // constant): load it (16 KB at N = 1024) instead of 1024 sincos per
  // workgroup.  tab_prev is a word no workgroup of this launch writes, so
  // every workgroup takes the same branch.
  const bool cached = pa.tab_prev != nullptr && *pa.tab_prev == Pc0;
  // (sin, cos)(t_i DAY 2pi/Pc0) for i = first, first + stride, ... < n, into
  // LDS; this workgroup's slice [lo, hi) of the cadences also to the global table
  auto table = [&](int first, int stride) {
    if (cached) {
      for (int i = first; i < n; i += stride) tabl[i] = pa.ph[i];
    } else {
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
    }
    if (blockIdx.x == 0 && first == 0 && pa.tab_mark != nullptr) *pa.tab_mark = Pc0;
  };
  __syncthreads();
  HB_PCLK(1, 0);
  auto none = []() {};
  if constexpr (WPB > kPrepRoles) {
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
      if (i < nb * kWcDoubles) reinterpret_cast<double*>(pa.wc)[(size_t)base * kWcDoubles + i] = v[u];
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // the stores acknowledged (L2) before any wave's scalar loads
  __syncthreads();
  HB_PCLK(3, 0);
}

// One wave per walker (WPB walkers per workgroup, one wave each; a wave's LDS
// is its lds_per-byte slice; the waves of a workgroup meet only in the fused
// prologue, everything else syncs per wave: HB_WSYNC).
// ACC (device sampler): the wave then runs the Hastings test and history write
// of its slot (hb_accept.hpp) on the logL it just computed, in place of a
// separate ds_accept launch; its operands are loaded when the wave starts.
// WPW = 2 / 4: a pair (four) of waves per walker (N = 1281..4096, see
// PairShared): wave h owns lane rows 64 h .. 64 h + 63 of 64 WPW; VPT is then
// the cadences per lane of the walker's rows (<= 16).
// PRE: the fused launch (fused_prologue above): WPB walkers per workgroup, the
// records computed in the prologue, the phase table read from LDS.
template <int VPT, bool ACC = false, int WPB = 1, int WPW = 1, bool PRE = false>
__global__ __launch_bounds__(64 * WPB * WPW) HB_WPE_ATTR void hb_eval_wave_kernel(
    const double* __restrict__ t, const double2* __restrict__ ph, const double* __restrict__ f,
    const double* __restrict__ isg, const double* __restrict__ rows,
    long n, long kth, const WalkerConst* __restrict__ wcs, double* __restrict__ logl,
    double* __restrict__ tmpl_out, int mode, int slab_bytes, double gap, hbds::AccArgs hst, int count, int lds_per,
    double* __restrict__ dqbuf, PreArgs pre) {
  static_assert(WPW == 1 || (WPW <= kMaxWPW && WPB == 1 && !ACC), "pair/rows: plain batched path");
  static_assert(!PRE || (WPW == 1 && !ACC && WPB >= kPrepRoles), "fused launch: plain one-wave batched path");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_all[];
  const int lane = threadIdx.x & 63;
  const int wib = WPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int slot = (int)blockIdx.x * WPB + wib;
  const bool valid = WPB == 1 || slot < count;
  unsigned char* smem = smem_all + (size_t)wib * (size_t)lds_per;
  if constexpr (PRE) {
    double2* tabl = reinterpret_cast<double2*>(smem_all + (size_t)WPB * (size_t)lds_per);
    fused_prologue<WPB>(pre, count, (int)n, t, smem_all, tabl);
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
  if (ACC && hst.ecnt_next != nullptr && slot == 0 && lane < hbds::kOrdBins)
    hst.ecnt_next[lane * hbds::kEbinStride] = 0;  // the next iteration's e-bin counters
  if (!valid) return;
  // the select's survivors: past the slab, or (fused launch) inside it, past
  // the histogram (the slab is dead once the keys are in registers)
  const int cand_off = PRE && slab_bytes >= kCandInSlab ? (4 << kSelBits) : slab_bytes;
  eval_wave_body<VPT, ACC, WPW>(t, ph, f, isg, rows, n, kth, wcs[wv], wv, slot, logl, tmpl_out, mode, slab_bytes,
                                cand_off, gap, hst, smem, dqbuf);
}

// ---------------------------------------------------------------------------
// The catalog's eval launch (CatSegs, hb_internal.hpp): every size class in
// one grid, largest walkers first.  Workgroups start in grid order as earlier
// ones retire, so the short walkers of the later segments fill the SIMDs the
// long ones leave idle while they drain -- no per-class launches, no streams
// or events between them.  128 threads per workgroup in every segment (two
// one-wave walkers, or a pair of waves for one walker), so the launch's one
// LDS size fits eight workgroups, four waves per SIMD, on a CU.
// ---------------------------------------------------------------------------
template <int VPT, int WPW>
__device__ __forceinline__ void cat_walker(const double* __restrict__ t, const double2* __restrict__ ph,
                                           const double* __restrict__ f, const double* __restrict__ isg,
                                           const double* __restrict__ rows, const TargetDesc& td,
                                           const WalkerConst& w, int wv, int pos, double* __restrict__ logl,
                                           int slab, unsigned char* smem, double* dq) {
  eval_wave_body<VPT, false, WPW>(t + td.off, ph + td.off, f + td.off, isg + td.off, rows + td.roff, td.n, td.kth, w,
                                  wv, pos, logl, nullptr, 0, slab, slab, td.gap, hbds::AccArgs{}, smem, dq);
}
// Each wave reads its CatJob row (catalog_layout), its target's TargetDesc and
// its walker's record through constant-address-space pointers: scalar loads
// at the use, nothing indexed at run time in the kernel arguments (the round-5
// CatSegs argument, indexed by the segment, held 262 SGPR spills).
__global__ __launch_bounds__(128) HB_WPE_ATTR void hb_eval_catalog_kernel(
    const CatJob* __restrict__ jobs, const double* __restrict__ t, const double2* __restrict__ ph,
    const double* __restrict__ f, const double* __restrict__ isg, const double* __restrict__ rows,
    const TargetDesc* __restrict__ tab, const WalkerConst* __restrict__ wcs, double* __restrict__ logl,
    unsigned char* __restrict__ dqb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_all[];
  typedef const __attribute__((address_space(4))) CatJob cjob_t;
  typedef const __attribute__((address_space(4))) TargetDesc ctd_t;
  typedef const __attribute__((address_space(4))) WalkerConst cwc_t;
  const int h = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const CatJob* jb = (const CatJob*)(cjob_t*)jobs;
  const CatJob& j = jb[2 * (int)blockIdx.x + h];
  const int wv = j.wv;
  if (wv < 0) return;
  const TargetDesc& td = ((const TargetDesc*)(ctd_t*)tab)[j.tgt];
  const WalkerConst& w = ((const WalkerConst*)(cwc_t*)wcs)[wv];
  const int geo = j.geo;
  unsigned char* smem = smem_all + ((geo >> 8) == 2 ? 0 : h * j.lds_per);
  double* dq = reinterpret_cast<double*>(dqb + j.dq);
  const int slab = j.slab, pos = j.pos;
  switch (geo) {
    case 16 | 2 << 8: cat_walker<16, 2>(t, ph, f, isg, rows, td, w, wv, pos, logl, slab, smem, dq); break;
    case 16 | 1 << 8: cat_walker<16, 1>(t, ph, f, isg, rows, td, w, wv, pos, logl, slab, smem, dq); break;
    case 8 | 1 << 8: cat_walker<8, 1>(t, ph, f, isg, rows, td, w, wv, pos, logl, slab, smem, dq); break;
    case 4 | 1 << 8: cat_walker<4, 1>(t, ph, f, isg, rows, td, w, wv, pos, logl, slab, smem, dq); break;
    case 2 | 1 << 8: cat_walker<2, 1>(t, ph, f, isg, rows, td, w, wv, pos, logl, slab, smem, dq); break;
    default: cat_walker<1, 1>(t, ph, f, isg, rows, td, w, wv, pos, logl, slab, smem, dq); break;
  }
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
    // neighbouring cadences mostly share a bin: add each run of equal bins
    // (within a row of 16 lanes: DPP row_shr:1 compares with lane-1) once,
    // from its first lane, instead of up to 64 same-address LDS atomics
    // (N = 20 000: 1.18 -> 1.04 ms per step, round 2)
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

// first digit of the block select: 10 bits like the one-wave kernels (C3 at
// 9 / 11 / 12 bits: +0.8% / -0.2% / +0.5% per step, profiles/r05/r05q_c3_sel_bits_ab.txt)
constexpr int kBlkSelBits = kSelBits;
template <int NW, int VPT>
__device__ double block_select2(const uint64_t (&key)[VPT], uint32_t kth, uint64_t kmin, uint64_t kmax,
                                uint32_t* hist, uint64_t* cand, SelShared* sh) {
  const int tid = threadIdx.x;
  if (kmin == kmax) return dval(kmin);
  int hi = 63 - __builtin_clzll(kmin ^ kmax);
  uint64_t mask = (hi == 63) ? 0ull : ~((2ull << hi) - 1ull);
  uint64_t prefix = kmin & mask;
  uint32_t kk = kth, cnt = 0;
  block_select_pass<NW, VPT, kBlkSelBits>(key, hist, sh, tid, hi, mask, prefix, kk, cnt);
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
  uint64_t* cand = reinterpret_cast<uint64_t*>(smem + sizeof(SelShared) + (4u << kBlkSelBits));
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wv = blockIdx.x;
  const WalkerConst& w = wcs[wv];
  double ll0;
  if (mode == 0 && logl_without_light_curve(w, ll0)) {  // see hb_eval_kernel
    if (tid == 0) logl[wv] = ll0;
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
  const double med = block_select2<NW, VPT>(key, (uint32_t)kth, kmn, kmx, hist, cand, sh);
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

// Kepler probe (tests/test_gpu_parity.py::test_kepler_cold_start_against_
// reference_root): the cold path's start and Newton loop exactly as the eval
// kernels run them -- cold_start_k (the fifth-order series start when the
// walker is on the phase table and |e| <= kSeriesEmax, else the reference's
// E0 = M + 0.85 e sign(sin M), likelihood3.c:155-157) then newton_k with its
// stopping rule -- one lane per mean anomaly M in (-2pi, 2pi) \ {0} (what
// mean_anomaly_k hands over), the table entry (sin, cos)(M) as the prep kernel
// writes it (psi = 0).  out[4 i ..] = {E, converged, sin E, cos E}.
__global__ void hb_kepler_probe_kernel(const double* __restrict__ M, long n, double e, int tab,
                                       double* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  WalkerConst w = {};
  w.e = e;
  w.e085 = 0.85 * e;
  w.cpsi = 1.0;
  w.spsi = 0.0;
  sincos_table(0.85 * e, w.sdel, w.cdel);
  w.mA = 1.0;
  double m[1] = {act ? M[i] : 1.0};
  const double t[1] = {m[0] / kDay};  // read only on lanes flagged exact: none here
  const bool plus[1] = {(fabs(m[0]) <= kPi) != (m[0] < 0.0)};
  double2 ph[1];
  sincos_table(m[0], ph[0].x, ph[0].y);
  double E[1], sv[1], cv[1], yk[1];
  bool ok = true;
  cold_start_k<1>(t, ph, tab != 0, false, w, m, plus, E, sv, cv, ok);
  const bool conv = newton_k<1>(e, m, E, sv, cv, yk, ok);
  if (act) {
    out[4 * i] = E[0];
    out[4 * i + 1] = conv ? 1.0 : 0.0;
    out[4 * i + 2] = sv[0];
    out[4 * i + 3] = cv[0];
  }
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
                       double2* ph, const int* cw0, const int* wf, double* tab_pc) {
  if (nwalk <= 0) return hipSuccess;
  if (t == nullptr || (tab != nullptr && (cw0 == nullptr || wf == nullptr))) ph = nullptr;
  // the most walkers per workgroup that still leave >= 256 workgroups (one per CU),
  // at most 32: both stars' lane tasks then fit one pass (prep_records); 64
  // walkers (two passes) measured 0.1648 vs 0.1640 ms per C5 call
  // (profiles/r04/r04k_c5_w*.json, interleaved)
  static const int wmax = getenv("HB_PREP_WMAX") ? atoi(getenv("HB_PREP_WMAX")) : 32;  // A/B knob
  const int nw = (wmax >= 64 && nwalk >= 256 * 64) ? 64 : (wmax >= 32 && nwalk >= 256 * 32) ? 32 : kPrepWalkers;
  const int nb = (nwalk + nw - 1) / nw;
  auto kern = nw == 64 ? hb_prep_kernel<64> : nw == 32 ? hb_prep_kernel<32> : hb_prep_kernel<kPrepWalkers>;
  hipLaunchKernelGGL(kern, dim3(nb), dim3(kPrepThreads), 0, s, d_params, nwalk, ma, d_wc, tab, wt, t,
                     (int)n, ph, cw0, wf, tab_pc);
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

constexpr size_t kLdsCap = 163840;

template <int VPT, bool ACC, int WPB, int WPW = 1, bool PRE = false>
static hipError_t launch_wave_g(size_t lds_per, int count, hipStream_t s, const double* t, const double2* ph,
                                const double* f, const double* sg, const double* rows, long n, long kth, const WalkerConst* wc,
                                double* logl, double* tmpl, int mode, size_t slab, double gap,
                                const hbds::AccArgs& acc, double* dq, const PreArgs* pre = nullptr) {
  auto kern = hb_eval_wave_kernel<VPT, ACC, WPB, WPW, PRE>;
  // PRE: the slices, then the LDS phase table (16 B per cadence)
  const size_t lds = (size_t)WPB * lds_per + (PRE ? (((size_t)n * 16 + 15) & ~(size_t)15) : 0);
  if (lds > kLdsCap) return hipErrorInvalidValue;
  static bool attr_set = false;  // per instantiation; benign race (idempotent)
  if (!attr_set && lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsCap);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((count + WPB - 1) / WPB), dim3(64 * WPB * WPW), lds, s, t, ph, f, sg, rows, n, kth, wc, logl,
                     tmpl, mode, (int)slab, gap, acc, count, (int)lds_per, dq, pre ? *pre : PreArgs{});
  return hipGetLastError();
}

// LDS bytes per walker of the fused launch: the slab, with the survivors
// inside it when it is big enough (kCandInSlab)
static size_t fused_lds_per(const EvalPlan& pl) {
  const size_t slab = pl.slab_bytes;
  return slab >= (size_t)kCandInSlab ? slab : wave_lds_bytes(slab, pl.vpt, 1);
}

// the prologue's scratch (prep records), which aliases the workgroup's slabs
static size_t fused_scratch_bytes(int wpb) {
  return wpb == 16 ? sizeof(PrepShared<16>) : wpb == 8 ? sizeof(PrepShared<8>) : sizeof(PrepShared<4>);
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
  if (mode == 0 || pl.vpt <= 0 || pl.vpt > 16 || pl.wpw != 1) return 0;
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
    return launch_wave_g<VPT, false, WV, 1, true>(per, nwalk, s, t, pa.ph, f, sg, rows, pl.n, pl.kth, pa.wc, logl, \
                                                  nullptr, 0, pl.slab_bytes, pl.gap, none, dq, &pa);
  HB_FCASE(16)
  HB_FCASE(8)
  HB_FCASE(4)
#undef HB_FCASE
  return hipErrorInvalidValue;
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

// one walker per workgroup (WPW waves)
template <int VPT, bool ACC, int WPW = 1>
static hipError_t launch_wave_w(size_t slab, int count, hipStream_t s, const double* t, const double2* ph,
                                const double* f, const double* sg, const double* rows, long n, long kth, const WalkerConst* wc,
                                double* logl, double* tmpl, int mode, double gap, const hbds::AccArgs& acc, double* dq) {
  const size_t per = wave_lds_bytes(slab, VPT, WPW);
  return launch_wave_g<VPT, ACC, 1, WPW>(per, count, s, t, ph, f, sg, rows, n, kth, wc, logl, tmpl, mode, slab, gap, acc,
                                         dq);
}

template <int VPT>
static hipError_t launch_wave_t(const EvalPlan& pl, const double* t, const double2* ph, const double* f,
                                const double* sg, const double* rows,
                                const WalkerConst* wc, int nwalk, double* logl, double* tmpl, int mode,
                                hipStream_t s, double* dq) {
#define HB_WPW_CASE(WV)                                                                                      \
  if (pl.wpw == WV)                                                                                          \
    return launch_wave_w<VPT, false, WV>(pl.slab_bytes, nwalk, s, t, ph, f, sg, rows, pl.n, pl.kth, wc, logl, tmpl, \
                                         mode, pl.gap, hbds::AccArgs{}, dq);
  if constexpr (VPT == 16 || VPT == 8) {
    HB_WPW_CASE(2)
  }
  if constexpr (VPT == 16) {
    HB_WPW_CASE(4)
  }
#undef HB_WPW_CASE
  if (pl.wpw != 1) return hipErrorInvalidValue;
  return launch_wave_w<VPT, false>(pl.slab_bytes, nwalk, s, t, ph, f, sg, rows, pl.n, pl.kth, wc, logl, tmpl, mode,
                                   pl.gap, hbds::AccArgs{}, dq);
}

template <int VPT>
static hipError_t launch_wave_acc_t(const EvalPlan& pl, const double* t, const double2* ph, const double* f,
                                    const double* sg, const double* rows, const WalkerConst* wc, int nwalk,
                                    double* logl, hipStream_t s, const hbds::AccArgs& acc, double* dq) {
  return launch_wave_w<VPT, true>(pl.slab_bytes, nwalk, s, t, ph, f, sg, rows, pl.n, pl.kth, wc, logl, nullptr, 0,
                                  pl.gap, acc, dq);
}

hipError_t launch_eval_catalog(const CatSegs& sg, const CatJob* jobs, const double* t, const double2* ph,
                               const double* f, const double* isg, const double* rows, const TargetDesc* tab,
                               const WalkerConst* wc, double* logl, unsigned char* dq, hipStream_t s) {
  if (sg.nseg <= 0 || sg.nseg > kCatSegs) return sg.nseg == 0 ? hipSuccess : hipErrorInvalidValue;
  size_t lds = 0;
  for (int q = 0; q < sg.nseg; ++q) {
    const bool ok1 = sg.wpw[q] == 1 && (sg.vpt[q] == 1 || sg.vpt[q] == 2 || sg.vpt[q] == 4 || sg.vpt[q] == 8 ||
                                        sg.vpt[q] == 16);
    const bool ok2 = sg.wpw[q] == 2 && sg.vpt[q] == 16;
    if (!(ok1 || ok2) || sg.first[q + 1] < sg.first[q] || sg.cnt[q] < 0) return hipErrorInvalidValue;
    if ((long)sg.first[q + 1] - sg.first[q] != (sg.wpw[q] == 2 ? (long)sg.cnt[q] : ((long)sg.cnt[q] + 1) / 2))
      return hipErrorInvalidValue;
    if ((size_t)sg.lds_per[q] < wave_lds_bytes((size_t)sg.slab[q], sg.vpt[q], sg.wpw[q])) return hipErrorInvalidValue;
    lds = std::max(lds, (size_t)sg.lds_per[q] * (sg.wpw[q] == 2 ? 1 : 2));
  }
  if (sg.first[0] != 0 || sg.first[sg.nseg] <= 0) return sg.first[sg.nseg] == 0 ? hipSuccess : hipErrorInvalidValue;
  if (lds > kLdsCap) return hipErrorInvalidValue;
  static bool attr_set = false;  // benign race (idempotent)
  if (!attr_set && lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&hb_eval_catalog_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsCap);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(hb_eval_catalog_kernel, dim3(sg.first[sg.nseg]), dim3(128), lds, s, jobs, t, ph, f, isg, rows,
                     tab, wc, logl, dq);
  return hipGetLastError();
}

hipError_t launch_eval(const EvalPlan& pl, const double* t, const double2* ph, const double* f, const double* sg,
                       const double* rows, const WalkerConst* wc, int nwalk, double* logl, double* tmpl, double* scratch,
                       int mode, hipStream_t s, const hbds::AccArgs* acc, double* dq) {
  if (nwalk <= 0) return hipSuccess;
  if (pl.vpt > 0 && dq == nullptr) return hipErrorInvalidValue;  // the one-wave path's deferred queue
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
  // the template in LDS always takes the register-key block kernel above; the
  // LDS-walking select of hb_eval_kernel keeps light curves whose template
  // does not fit LDS (N > 20 300), in an HBM slab
  if (pl.lds) return hipErrorInvalidValue;
  switch (pl.nw) {
    case 1: return launch_eval_t<1, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
    case 2: return launch_eval_t<2, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
    case 4: return launch_eval_t<4, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
    case 8: return launch_eval_t<8, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
    case 16: return launch_eval_t<16, false>(pl, t, ph, f, sg, wc, nwalk, logl, tmpl, scratch, mode, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_traj(const double* d_times, int nt, const TrajArgs& ta, double* d, double* z1,
                       double* z2, double* rr, double* ff, hipStream_t s) {
  if (nt <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb_traj_kernel, dim3((nt + 255) / 256), dim3(256), 0, s, d_times, nt, ta, d, z1, z2,
                     rr, ff);
  return hipGetLastError();
}

hipError_t launch_kepler_probe(const double* d_m, long n, double e, int tab, double* d_out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(hb_kepler_probe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d_m, n, e, tab, d_out);
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
constexpr long kPairNmin = 64 * 20 + 1;  // smallest N of the pair plan
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
size_t wave_slab_bytes(long n, long nr) {
  if (nr <= 0) nr = wave_nr_for(n);
  const int rc = (int)((n + nr - 1) / nr);
  const long live = (n + rc - 1) / rc;
  int stride = rows_stride(rc);
  if (nr > 128 && live * stride * 8 > kRowsLdsCap) stride = rc;  // as make_rows
  const size_t vals = (size_t)(nr > 128 ? live : nr) * stride * 8;
  const size_t slab = vals > (size_t)(4u << kSelBits) ? vals : (size_t)(4u << kSelBits);
  return (slab + 15) & ~(size_t)15;
}

// bytes of the one-wave kernel's deferred queue for `count` walkers of wpw
// waves
size_t wave_queue_bytes(int vpt, long count, int wpw) {
  return (size_t)count * (size_t)wpw * ((size_t)64 * (size_t)vpt + kDqSink) * 16;
}

// slab | select candidates | eclipse queue (chain model pass only) | the
// pair's shared words (wpw = 2)
size_t wave_lds_bytes(size_t slab, int vpt, int wpw) {
  (void)vpt;
  const size_t cb = 8 * (size_t)kCandMax;
  return (slab + cb + (wpw > 1 ? sizeof(PairShared) : 0) + 15) & ~(size_t)15;
}

// t, f and 1/sigma in the one-wave kernel's lane-row order: row block c holds
// cadence l * rc + c for lane rows l = 0..nr-1 (nr = wave_nr_for(n), rc =
// ceil(n / nr); cadences past the end repeat the last one and are never used)
long wave_rows_doubles(long n, long nr) {
  if (nr <= 0) nr = wave_nr_for(n);
  return 3L * nr * ((n + nr - 1) / nr);
}
void build_rows(const double* t, const double* f, const double* isg, long n, double* out, long nr) {
  if (nr <= 0) nr = wave_nr_for(n);
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
  if (wave_nr_for(n) > 0) {  // one wave (or 2..16) per walker, keys in registers
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
    const long per = (n + 64L * nw - 1) / (64L * nw);  // cadences per thread
    if (per <= 32 && need >= sizeof(SelShared) + (4u << kBlkSelBits) + 8 * kCandMax)
      // exact fit at 17..20 (C3: N = 20 000 over 16 waves is 19.5 per thread): 24
      // key slots there cost <16, 24> 14 VGPR spills (64 B of scratch per lane).
      // Whenever the slab fits LDS, per <= 20 (N <= 20 300 over 16 waves; fewer
      // waves only for shorter light curves), so 24 / 32 keys are never needed
      // (and not instantiated: they spill)
      pl.bvpt = per <= 8 ? 8 : per <= 16 ? 16 : per <= 20 ? 20 : 0;
  } else {
    pl.lds = false;
    pl.lds_bytes = sizeof(SelShared);
    pl.nw = 4;
  }
  return pl;
}

}  // namespace hbk

#ifdef HB_WAVE_CLOCKS
extern "C" int hb_debug_prologue_clocks(unsigned long long* out, int nwg) {
  if (nwg > 4096) nwg = 4096;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hb_pro_clk), 16 * sizeof(unsigned long long) * nwg);
  return e == hipSuccess ? 0 : -1;
}
extern "C" int hb_debug_wave_clocks(unsigned long long* out, int nwaves) {
  if (nwaves > 65536) nwaves = 65536;
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hb_wave_clk), kClkWords * sizeof(unsigned long long) * nwaves);
  return e == hipSuccess ? 0 : -1;
}
#endif
