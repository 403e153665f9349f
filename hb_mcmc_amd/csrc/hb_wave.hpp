// hb_wave.hpp -- the one-wave-per-walker likelihood (N <= 2048 per wave; 2 or
// 4 waves per walker up to 4096) as device functions: lane-row model passes
// (warm Kepler chains or the cold sweep), the deferred eclipse / slow-path
// queue, exact median by register-key radix select, chi^2 and the Gaia /
// Roche terms (likelihood3.c:530-686, 86-105, 809-873), and the fused
// Hastings test (hb_accept.hpp).  Shared by the batched eval kernels
// (hb_kernels.hip hb_eval_wave_kernel, hb_eval_catalog_kernel), which call
// eval_wave_body() once the walker's record (WalkerConst) is in memory.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hb_accept.hpp"
#include "hb_device.hpp"
#include "hb_internal.hpp"

// per-wave shader clocks: hb_kernels.hip defines these under HB_WAVE_CLOCKS
// (experiment builds); no-ops otherwise
#ifndef HB_CLK_BEGIN
#define HB_CLK_BEGIN() do { } while (0)
#define HB_CLK_MARK(i) do { } while (0)
#define HB_CLK_END(wv) do { } while (0)
#endif

// LDS ordering among the lanes of ONE wave (the one-wave-per-walker kernel may
// share its workgroup with other walkers' waves, which must not be waited for)
#define HB_WSYNC()                                        \
  do {                                                    \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
    __builtin_amdgcn_wave_barrier();                      \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
  } while (0)
namespace hbk {

using namespace hbdev;

constexpr int kK = 4;  // cadences interleaved per lane in the cold model loop (4: +1% over 2 on MI355X)

// One-wave kernel: lane l owns the rc = ceil(n/64) consecutive cadences
// l*rc .. l*rc + rc - 1 (its row of the LDS slab, later its select keys).
// The chain path solves a row as KC chains whose Kepler starts are warm
// (chain_kepler_warm) after each chain's first cadence.  Row stride rc | 1:
// an odd stride spreads a wave's accesses at one row position over the banks,
// and position c of a lane's row sits at a constant offset from the row's
// start, so the key loads take immediate offsets (no per-key address
// arithmetic).  The slab is ~n * 8 bytes, so short light curves of a catalog
// class keep more waves per CU.
#ifndef HB_KC
#define HB_KC 2  // Kepler chains per lane (KC = 4: 108 VGPR spills, C2 eval 48.9 vs 38.7 us, profiles/r05/r05a_kc4_ab.txt)
#endif
struct Rows {
  int rc;      // cadences per lane row
  int stride;  // row stride [doubles]
  float rcp;   // 1 / rc (row of cadence i, i < 2^11: exact after rounding)
  int live;    // rows holding cadences: ceil(n / rc) (the rows kernel stores no others)
};
constexpr long kRowsLdsCap = 163840 - 2048;  // the rows kernel's slab, below its candidates and shared words
__host__ __device__ __forceinline__ int rows_stride(int rc) { return rc | 1; }
// nr lane rows per walker: 64 (one wave), 128 (a pair of waves, WPW = 2) or
// 256 (four waves)
__device__ __forceinline__ Rows make_rows(int n, int nr = 64) {
  Rows r;
  r.rc = (n + nr - 1) / nr;
  r.stride = rows_stride(r.rc);
  r.live = (n + r.rc - 1) / r.rc;
  // many rows (the rows kernel, nr > 128): the odd pad only while the live rows fit the LDS
  if (nr > 128 && (long)r.live * r.stride * 8 > kRowsLdsCap) r.stride = r.rc;
  r.rcp = 1.0f / (float)r.rc;
  return r;
}
__device__ __forceinline__ int slab_pos(const Rows& r, int lane, int c) { return lane * r.stride + c; }
// slab position of cadence i: row q = i / rc by the fp32 reciprocal
// ((i + 0.5) / rc is >= 1/(2 rc) away from an integer, far above its error)
__device__ __forceinline__ int slab_pos_of(const Rows& r, int i) {
  const int q = (int)(((float)i + 0.5f) * r.rcp);
  return slab_pos(r, q, i - q * r.rc);
}

// Deferred cadence queue: the model pass writes every cadence's polynomial
// value to the slab and appends the cadences that need more to a per-wave
// region of global memory -- eclipsing ones (dd with the sign of zz, slab
// position) and the rare ones outside the fast sincos/fmod domain (slab
// position | kSlowFlag).  Eclipse terms are rare and spread over the orbit, so
// inline terms would run the overlap area for a few lanes at almost every
// step; after the pass, 64 entries at a time, the eclipse term (inlined) is
// subtracted from the slab value -- the same v - term as inline -- and
// slow-path cadences are recomputed in reference order.  The model loop then
// holds no function call.  Capacity per wave: 64 VPT entries (every cadence,
// worst case) behind one 16-B sink entry.
constexpr int kSlowFlag = 1 << 30;
struct DeferQ {
  char* e;  // this wave's entries (the base is held in VGPRs: no SGPR spill reloads per push)
  int n;    // entries (wave-uniform)
};
// entries in front of a wave's region: the sink
constexpr int kDqSink = 1;
// One 16-B entry per queued cadence: (dd with the sign of zz, code = slab
// position | kSlowFlag for the slow path); one store, one load.  The push is
// branch-free: lanes that queue nothing store into the wave's sink entry (the
// 16 B in front of its region, never read), so the model pass's step stays one
// basic block that the scheduler can interleave.
__device__ __forceinline__ void dq_push(DeferQ& q, bool push, double a, int code) {
  const unsigned long long bal = wave_ballot(push);
  // global address space spelled out (the VGPR base hides it from inference)
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(1))) d2v gdouble2;
  const uint32_t pos = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)bal, (unsigned)q.n));
  const d2v ent = {a, __longlong_as_double((long long)code)};
  const long off = push ? (long)pos << 4 : -16L;
  *(gdouble2*)(q.e + off) = ent;
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
// cadence spacing, host-side), at most kWarmD1.  Steps that miss the one-step
// fast path continue with the Newton loop from the warm iterate, which still
// takes fewer steps than the reference's start; past the gate (sparse or
// shuffled cadences) the cold path with four interleaved cadences per lane is
// faster.
#ifndef HB_WARM_D1
#define HB_WARM_D1 0x1p-4  // A/B knob (2^-10 until round 5: profiles/r05/r05za_warm_gate_ab.txt)
#endif
constexpr double kWarmD1 = HB_WARM_D1;
// cadences per lane of the chain path (4: catalog classes of 129-256 cadences
// on warm chains measured within noise, profiles/r05/r05c_c5_ab.txt)
constexpr int kChainVptMin = 8, kChainVptMax = 32;
__device__ __forceinline__ bool chain_eligible(const WalkerConst& w, double gap) {
  const double e = fabs(w.e);  // e < 0 is Kepler's equation at M + pi, E + pi
  const double dm = gap * kDay * fabs(w.mA);
  const double ome = 1.0 - e;
  return (e <= kWarmEmax) && (e * dm * dm <= 2.0 * kWarmD1 * ome * ome * ome);
}

// Wave pacing.  The waves sharing a SIMD are issued by priority, then age:
// with equal priorities the oldest wave runs nearly unimpeded and finishes
// first, and the youngest runs its last stretch alone, latency-bound
// (scripts/wave_clocks.py: finish times 46k/69k/89k/107k cycles for the four
// waves of a SIMD at C2, round 2).  The pacer lowers a wave's priority by
// quartile of its own model pass (3 -> 0): mean resident waves 2.86 -> 3.32,
// -4%.  (Pacing by the lead over the slowest wave of the same SIMD, progress
// words in LDS, kept 3.6 waves resident but did not run faster: round 2.)
struct Pacer {
  int q1, q2, q3;  // first steps of the 2nd, 3rd and 4th quarter
  __device__ __forceinline__ void begin(int steps) {
    q1 = (steps + 3) >> 2;
    q2 = (steps + 1) >> 1;
    q3 = (3 * steps + 3) >> 2;
  }
  __device__ __forceinline__ void step(int j) const {
    if (j == q1) __builtin_amdgcn_s_setprio(2);
    if (j == q2) __builtin_amdgcn_s_setprio(1);
    if (j == q3) __builtin_amdgcn_s_setprio(0);
  }
};

// Cold path in the one-wave kernel: the wave sweeps the light curve 64*K
// consecutive cadences at a time (cadence base + k*64 + lane), so the eclipse
// lanes of an iteration are neighbours in phase.  Values are stored at the
// lane-row slab positions (slab_pos_of) that the key load reads; eclipsing
// and slow-path cadences go to the deferred queue.
// NT threads per walker (64, or 128 for a pair of waves), thread tid; K
// interleaved cadences per lane (at most the walker's cadences per lane: a
// 2-per-lane light curve runs 2, not 4 with two of them padding)
template <int NT = 64, int K = kK>
__device__ __forceinline__ void model_pass_cold(const double* __restrict__ t, const double2* __restrict__ ph,
                                                int n, const Rows& rw, const WalkerConst& w, double* vals,
                                                int lane, Pacer pc, DeferQ& dq) {
  const bool tab = (ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  const int last = n - 1;
  const int nit = (n + K * NT - 1) / (K * NT);
  pc.begin(nit);
  for (int base = 0, it = 0; base < n; base += K * NT, ++it) {
    pc.step(it);
    double tk[K], v[K];
    double2 pk[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = min(base + k * NT + lane, last);
      tk[k] = t[i];
      pk[k] = tab ? ph[i] : make_double2(0.0, 1.0);
    }
    bool bad;
    __asm__ volatile("" ::: "memory");
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
  }
}

// Software-pipelined chain model pass: the loop body of step j holds step j's
// warm Kepler solve and step j-1's polynomial, which both read only the chain
// state left by step j-1 -- one basic block with two independent dependency
// chains per Kepler chain (ILP 2 KC instead of KC for the latency-bound tail
// of the launch).  Step j-1's values are stored and queued after it, then
// step j is finished (converged lanes: the reciprocal; else the general
// Newton loop / the reference's start).
// tT: the light curve's times in lane-row order (tT[c * NR + l] = t[l * rc + c],
// build_rows), so the step-c loads of the 64 lanes are one coalesced 512-B
// request instead of 64 strided ones.  NR: lane rows of the walker (the
// arrays' pitch: 64, or 128 / 256 for 2 / 4 waves, each passing tT offset by
// its first row); row: this lane's row.
template <int VPT>
constexpr int chain_kc() { return VPT < HB_KC ? VPT : HB_KC; }
// The chains' first cadences (step 0 of model_pass_chain_pipe): the
// reference's start from the phase-table entries, Newton to convergence.
template <int VPT, int NR = 64>
__device__ __forceinline__ void chain_step0(const double* __restrict__ tT, const double2* __restrict__ ph, int n,
                                            const Rows& rw, const WalkerConst& w, int lane, int row,
                                            ChainState<chain_kc<VPT>()>& st, bool& ok) {
  constexpr int KC = chain_kc<VPT>();
  const int lc = (rw.rc + KC - 1) / KC;
  const bool tab = (ph != nullptr) && (w.tab != 0.0);  // walker-uniform
  const int last = n - 1;
  const int base = row * rw.rc;
  double tk[KC];
  double2 p0[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) tk[k] = tT[min(k * lc, rw.rc - 1) * NR + lane];
#pragma unroll
  for (int k = 0; k < KC; ++k) p0[k] = tab ? ph[min(base + k * lc, last)] : make_double2(0.0, 1.0);
  ok = true;
  chain_first<KC>(tk, p0, tab, w, st, ok);
}
template <int VPT, int NR = 64>
__device__ __forceinline__ void model_pass_chain_pipe(const double* __restrict__ tT, const double2* __restrict__ ph,
                                                      int n, const Rows& rw, const WalkerConst& w, double* vals,
                                                      int lane, int row, Pacer pc, DeferQ& dq) {
  constexpr int KC = chain_kc<VPT>();
  const int lc = (rw.rc + KC - 1) / KC;  // chain length (wave-uniform)
  const int rs = row * rw.stride;  // slab_pos = rs + c
  const bool live = NR <= 128 || row < rw.live;
  ChainState<KC> st;
  double tk[KC];
  // the step whose polynomial is pending: its (s, c, 1/den) are the chain state
  bool pend_ok = true;
  chain_step0<VPT, NR>(tT, ph, n, rw, w, lane, row, st, pend_ok);
  // store the pending step jp's values and queue its eclipse / slow-path
  // cadences; cadences past n (the last row's padding) store harmless values
  // (their keys are masked); the rows kernel (NR > 128) sizes its slab to the
  // live rows and stores no others
  auto emit = [&](int jp, const double (&v)[KC], const double (&dd)[KC], const double (&zz)[KC], bool bad) {
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = k * lc + jp;
      if (c < rw.rc) {  // wave-uniform: the last chain may run past the row end
        const int sp = rs + c;
        if (live) vals[sp] = v[k];
        const bool need = (!bad) & eclipse_lane(w, dd[k], zz[k]);
        dq_push(dq, live & (bad | need), copysign(dd[k], zz[k]), sp | (bad ? kSlowFlag : 0));
      }
    }
  };
  const WarmK wk = warm_k(w.e);
  pc.begin(lc);
  for (int j = 1; j < lc; ++j) {
    pc.step(j);
    // the walker constants are reloaded (scalar loads) at every step instead
    // of being held in SGPRs across the loop: SGPR spills 138 -> 111 (fused
    // C2 kernel) and 206 -> 142 (device-sampler eval + Hastings), time
    // unchanged (profiles/r04/r04n_*.json)
    __asm__ volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < KC; ++k) tk[k] = tT[min(k * lc + j, rw.rc - 1) * NR + lane];
    double m[KC], E[KC], s[KC], c[KC], ys[KC], v[KC], dd[KC], zz[KC];
    bool ok = true, fine;
    chain_kepler_warm<KC>(tk, w, st, m, E, s, c, ys, fine, ok, wk);  // step j
    flux_poly_inv_k<KC>(st.s, st.c, st.inv, w, v, dd, zz);      // step j - 1, same block
    // the polynomial's values are materialised here, beside step j's solve:
    // otherwise the compiler sinks them into emit's conditional blocks, after
    // the solve, and the two no longer interleave
#pragma unroll
    for (int k = 0; k < KC; ++k) __asm__ volatile("" : "+v"(v[k]), "+v"(dd[k]), "+v"(zz[k]));
    // step j - 1's stores and pushes after step j's finish: their branches
    // (the wave-uniform row test) then do not split the solve and polynomial
    const bool pbad = !pend_ok;
    chain_finish_warm<KC>(tk, w, wave_all(fine), fine, m, E, s, c, ys, ok, st);
    emit(j - 1, v, dd, zz, pbad);
    pend_ok = ok;
  }
  {  // the last step's polynomial
    double v[KC], dd[KC], zz[KC];
    flux_poly_inv_k<KC>(st.s, st.c, st.inv, w, v, dd, zz);
    emit(lc - 1, v, dd, zz, !pend_ok);
  }
}

// ---------------------------------------------------------------------------
// One-wave-per-walker path (N <= 64*VPT): keys in VGPRs, the LDS template slab
// reused as a histogram (11-bit first digit), exact rank among <= 64
// survivors.  kth is the 0-based rank of likelihood3.c:97-101.
// ---------------------------------------------------------------------------
// select digit widths: 10 bits first (the whole light curve), then 8 over the
// survivors of one bin (11 / 9 first bits measured slower, round 3)
constexpr int kSelBits = 10;
constexpr int kSelBits2 = 8;
constexpr int kCandMax = 64;  // survivors ranked directly (<= 64: one per lane; 32 / 16 measured neutral)
// slab bytes from which the fused launch keeps the survivors inside the slab
// (above the 2^kSelBits-bin histogram)
constexpr int kCandInSlab = (4 << kSelBits) + 8 * kCandMax;

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

// ---------------------------------------------------------------------------
// Keys, median and chi^2 of the one-wave kernels with few non-fp64
// instructions:
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

// Key slot v of `lane` holds cadence lane*rc + v (its own row; v >= rc is
// padding).  A light curve is smooth, so 64 consecutive cadences mostly share
// one histogram bin and a wave's LDS atomic would serialise on one address;
// lane-owned rows give each atomic instruction 64 cadences spread over the
// whole light curve.
__device__ __forceinline__ int key_index(const Rows& r, int v, int lane) { return lane * r.rc + v; }


// The likelihood of walker wv (record w) by its wave(s), after the record is
// in memory: model pass, deferred queue, keys, exact median, chi^2 (mode 0:
// logl[wv]; mode 1: the template tmpl_out[wv][0..n)), and with ACC the
// Hastings test of local slot wv (hb_accept.hpp) on the logL just computed.
// t, ph, f, isg: the light curve in cadence order (ph: its shared-period
// phase table, or null); rows: t, f, 1/sigma in lane-row order (build_rows);
// smem: this walker's LDS slice (slab, then survivors at cand_off, then the
// pair's shared words); dqbuf: the deferred queues, region `slot`.
// WPW > 1: called by each of the walker's WPW waves (wave h of the workgroup).
template <int VPT, bool ACC, int WPW>
__device__ __forceinline__ void eval_wave_body(const double* __restrict__ t, const double2* __restrict__ ph,
                                               const double* __restrict__ f, const double* __restrict__ isg,
                                               const double* __restrict__ rows, long n, long kth,
                                               const WalkerConst& w, int wv, int slot, double* __restrict__ logl,
                                               double* __restrict__ tmpl_out, int mode, int slab_bytes, int cand_off,
                                               double gap, const hbds::AccArgs& hst, unsigned char* smem,
                                               double* __restrict__ dqbuf) {
  constexpr int NR = 64 * WPW;  // lane rows per walker
  const int lane = threadIdx.x & 63;
  const int h = WPW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;  // wave of the pair
  const int row = h * 64 + lane;
  HB_CLK_BEGIN();
  __builtin_amdgcn_s_setprio(3);  // the pacer lowers it by quartile of the model pass
  double* vals = reinterpret_cast<double*>(smem);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);
  uint64_t* cand = reinterpret_cast<uint64_t*>(smem + cand_off);
  double ll0 = 0.0;
  const bool early_exit = mode == 0 && logl_without_light_curve(w, ll0);
  Pacer pc{0, 0, 0};
  // the Hastings test's operands (uniform values and the 21-coordinate rows):
  // loaded after the model pass, in flight through the select, so they hold
  // no registers across the model loop (profiles/r05/r05p_ds_lost_acc_ab.txt)
  hbds::AccPre apre{};
  if (ACC && early_exit) apre = hbds::accept_prefetch(hst, wv, lane);
  if (early_exit) {  // Roche overflow, |e| > 1: logl_without_light_curve (hb_device.hpp)
    if (row == 0) logl[wv] = ll0;
    if (ACC) (void)hbds::accept_slot_wave_pre(hst, wv, ll0, lane, apre);
    HB_CLK_END(wv);
    return;
  }

  uint64_t key[VPT];
  const Rows rw = make_rows((int)n, NR);
  // t, f and 1/sigma in lane-row order (pitch NR), from this wave's first row
  const double* __restrict__ tT = rows + h * 64;
  const double* __restrict__ fT = rows + NR * rw.rc + h * 64;
  const double* __restrict__ iT = rows + 2 * NR * rw.rc + h * 64;
  PairShared* ps = reinterpret_cast<PairShared*>(smem + slab_bytes + 8 * kCandMax);  // WPW > 1 only
  // this wave's region of the deferred queue (64 VPT entries of 16 B)
  DeferQ dq{nullptr, 0};
  dq.e = reinterpret_cast<char*>(dqbuf) + ((size_t)slot * WPW + (size_t)h) * (size_t)((64 * VPT + kDqSink) * 16) +
         kDqSink * 16;
  __asm__ volatile("" : "+v"(dq.e));  // a VGPR pair, not one more scalar to spill
  if (VPT >= kChainVptMin && VPT <= kChainVptMax && chain_eligible(w, gap))
    model_pass_chain_pipe<VPT, NR>(tT, ph, (int)n, rw, w, vals, lane, row, pc, dq);
  else
    model_pass_cold<NR, (VPT < kK ? VPT : kK)>(t, ph, (int)n, rw, w, vals, row, pc, dq);
  HB_CLK_MARK(3);
  HB_WSYNC();  // the slab values of every lane are in place
  // a pair's cold pass writes cadences of either wave's rows, and its queued
  // eclipse terms land there too: the pair meets before and after them
  if (WPW > 1) __syncthreads();
  dq_apply(w, vals, dq, t, rw, (int)n, lane);
  if (WPW > 1) __syncthreads();
  if (ACC) apre = hbds::accept_prefetch(hst, wv, lane);
  HB_CLK_MARK(0);
  HB_WSYNC();
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
  if (ACC) (void)hbds::accept_slot_wave_pre(hst, wv, -c / 2.0, lane, apre);  // c is wave-uniform (readlanes)
  HB_CLK_END(wv);
}

}  // namespace hbk
