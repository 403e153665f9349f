// hb_internal.hpp -- types shared between the kernels and the host C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "hb_device.hpp"

namespace hbds {
struct AccArgs;
}

namespace hbk {

struct MagArgs {
  double mag[5];     // {D [pc], G, B-V, V-G, G-T}
  double magerr[4];
};

// LDS scratch of the eval kernel (precedes the template slab); 16-B multiple.
struct alignas(16) SelShared {
  uint32_t hist[256];
  unsigned long long red_min[16];
  unsigned long long red_max[16];
  double red_sum[16];
  unsigned long long ans;
  int bin;
  uint32_t before;
  uint32_t cnt;
  uint32_t ncand;  // survivor counter of the register-key block select
  uint32_t pad[2];
};
static_assert(sizeof(SelShared) % 16 == 0, "LDS carve must stay 16-B aligned");

struct EvalPlan {
  long n = 0;
  long kth = 0;        // 0-based rank of the subtracted "median"
  int nw = 1;          // waves per walker
  int vpt = 0;         // >0: one-wave path, cadences per lane (register keys)
  int wpw = 1;         // one-wave path: waves per walker (2: a pair, 1024 < n <= 2048)
  int bvpt = 0;        // >0: NW-wave path with register keys, cadences per thread
  size_t slab_bytes = 0;  // template slab / histogram bytes (one-wave path)
  bool lds = true;     // template in LDS (else HBM scratch slab)
  size_t lds_bytes = 0;
  double gap = 0.0;    // typical cadence spacing [d] (hb_cadence_gap), warm-chain gate
};

// One light curve of a catalog (hb_catalog_*): its slice of the concatenated
// t / f / (1/sigma) arrays and the magnitude data the Gaia term uses.
struct alignas(16) TargetDesc {
  long off;      // first cadence in the concatenated arrays
  long n;        // cadences (2..2048 in the batched path)
  long kth;      // 0-based median rank (likelihood3.c:97-99)
  long roff;     // first double of the target's lane-row arrays (build_rows)
  double dist;   // mag_data[0] [pc]
  double gmag;   // mag_data[1]
  double gerr;   // magerr[0]
  double gap;    // typical cadence spacing [d] (hb_cadence_gap), warm-chain gate
};

struct TrajArgs {
  hbdev::WalkerConst w;  // orbit fields only; aR carries a in cm
  double fz1, fz2;       // M2/Mtot, M1/Mtot after the traj() mass swap
};

enum ProbeOp {
  kOpAlphaBeam = 0,
  kOpBeaming,
  kOpEllipsoidal,
  kOpReflection,
  kOpEclipse,
  kOpGetT,
  kOpGetR,
  kOpEnvT,
  kOpEnvR,
  kOpRadiiTeffs,
  kOpMags,
  kOpRoche,
  kOpEggleton,
};

EvalPlan make_plan(long n);
// the multi-wave plan for any n (the batched path's choice above 2048 cadences,
// and the latency plan of small batches below)
EvalPlan make_block_plan(long n);
// 90th percentile of |t[i+1] - t[i]| (host; the eval kernel's warm-chain gate)
double cadence_gap(const double* t, long n);
// forces the load of hb_kernels.hip's code object on the current device
hipError_t preload_code_object();
// ph (optional): the shared-period phase table of the batch, (sin, cos)(t_i
// DAY 2pi/P) for P = the period of the light curve's first walker (walker 0,
// or in catalog mode the first walker of cadence i's target, cw0[i]; wf: each
// walker's target's first walker), written here and read by the eval launch;
// walkers with another period get tab = 0.  Catalog mode: n = all cadences.
hipError_t launch_prep(const double* d_params, int nwalk, const MagArgs& ma, hbdev::WalkerConst* d_wc,
                       hipStream_t s, const TargetDesc* tab = nullptr, const int* wt = nullptr,
                       const double* t = nullptr, long n = 0, double2* ph = nullptr, const int* cw0 = nullptr,
                       const int* wf = nullptr, double* tab_pc = nullptr);
// Catalog mode: ONE eval launch for every size class of the call.  Segment s
// of the grid (workgroups first[s] .. first[s+1]) evaluates the walkers
// list[off[s] .. off[s] + cnt[s]), each reading its target's slice through
// tab[wt[walker]]: wpw 1 -- two walkers per 128-thread workgroup, a wave each,
// vpt cadences per lane (64 lane rows); wpw 2 -- one walker per workgroup, a
// pair of waves of 16 cadences per lane (128 lane rows, N > 1024).
constexpr int kCatSegs = 6;
struct CatSegs {
  int nseg;
  int first[kCatSegs + 1];
  int vpt[kCatSegs];
  int wpw[kCatSegs];
  int off[kCatSegs];
  int cnt[kCatSegs];
  int slab[kCatSegs];     // slab bytes per walker
  int lds_per[kCatSegs];  // LDS bytes per walker (a wave's slice, or the pair's)
  long long dq[kCatSegs]; // byte offset of the segment's deferred queues in the dq buffer
};
// One wave's work in the catalog eval launch, built by catalog_layout from
// CatSegs: wave h of workgroup b reads job 2 b + h (a pair's two waves read
// the same walker).  Everything the wave needs besides its target's
// TargetDesc and its walker's record, in one 32-B row read by scalar loads --
// no segment search and no runtime-indexed kernel-argument arrays.
struct alignas(32) CatJob {
  int wv;         // walker (logL index); -1: nothing to do (the last one-wave workgroup's second wave)
  int tgt;        // its target (TargetDesc row)
  int pos;        // its position in the segment (deferred-queue region)
  int slab;       // slab bytes per walker
  long long dq;   // byte offset of the segment's deferred queues in the dq buffer
  int lds_per;    // LDS bytes per walker
  int geo;        // VPT | WPW << 8
};
static_assert(sizeof(CatJob) == 32, "CatJob layout");
hipError_t launch_eval_catalog(const CatSegs& sg, const CatJob* jobs, const double* t, const double2* ph,
                               const double* f, const double* isg, const double* rows, const TargetDesc* tab,
                               const hbdev::WalkerConst* wc, double* logl, unsigned char* dq, hipStream_t s);
// The fused launch: per-walker records (hb_prep.hpp) in the prologue of the
// one-wave eval kernel, WPB walkers per workgroup (hb_kernels.hip
// launch_eval_fused); the records and the shared-period phase table are also
// written to the context's buffers (as hb_prep_kernel writes them).
struct PreArgs {
  const double* params;     // W x 21
  MagArgs ma;
  hbdev::WalkerConst* wc;   // records out (then read back by the eval waves)
  double2* ph;              // the global phase table (each workgroup writes a slice)
  double* tab_pc;           // its period [s]
  // The previous fused launch's table period (a word only that launch wrote;
  // the host alternates two, hb_ctx::tab_seq), or null when another kernel
  // may have rewritten the table since: equal to this launch's P0, the global
  // table is complete for it and the prologue loads it instead of computing
  // it.  tab_mark: the word this launch writes for the next one.
  const double* tab_prev;
  double* tab_mark;
};
// walkers per workgroup of the fused launch for w walkers on `cus` CUs (0: the
// two-launch path: prep + eval)
int fused_wpb(const EvalPlan& pl, int w, int cus);
hipError_t launch_eval_fused(const EvalPlan& pl, int wpb, const PreArgs& pa, const double* t, const double* f,
                             const double* sg, const double* rows, int nwalk, double* logl, hipStream_t s, double* dq);
int wave_vpt_for(long n);  // cadences per lane of the one-wave path, 0 if n > 2048
int wave_nr_for(long n);   // lane rows per walker: 64, 128 (a pair of waves, 1280 < n <= 2048), 256 (four, <= 4096), 0 above
// device bytes of the one-wave kernel's deferred cadence queue for `count`
// walkers at `vpt` cadences per lane (the dq argument of launch_eval*)
size_t wave_queue_bytes(int vpt, long count, int wpw = 1);
size_t wave_slab_bytes(long n, long nr = 0);  // nr: lane rows (0: wave_nr_for(n))
size_t wave_lds_bytes(size_t slab, int vpt, int wpw = 1);
// t, f, 1/sigma in the one-wave kernel's lane-row order (3 x nr x ceil(n/nr) doubles)
long wave_rows_doubles(long n, long nr = 0);
void build_rows(const double* t, const double* f, const double* isg, long n, double* out, long nr = 0);
// acc (device sampler, one-wave path only): each wave also runs its slot's
// Hastings test and history write (hb_accept.hpp); hipErrorNotSupported on the
// multi-wave path
hipError_t launch_eval(const EvalPlan& pl, const double* t, const double2* ph, const double* f, const double* sg,
                       const double* rows, const hbdev::WalkerConst* wc, int nwalk, double* logl, double* tmpl,
                       double* scratch, int mode, hipStream_t s, const hbds::AccArgs* acc = nullptr,
                       double* dq = nullptr);
hipError_t launch_traj(const double* d_times, int nt, const TrajArgs& ta, double* d, double* z1,
                       double* z2, double* rr, double* ff, hipStream_t s);
hipError_t launch_probe(int op, const double* d_in, double* d_out, hipStream_t s);
hipError_t launch_kepler_probe(const double* d_m, long n, double e, int tab, double* d_out, hipStream_t s);
hipError_t launch_partition(double* d_a, int lo, int hi, int* d_res, hipStream_t s);
hipError_t launch_median(double* d_a, long n, long kth, hipStream_t s);
// ascending sort of d_in[0..n) into d_out (bitonic over order-preserving keys;
// d_keys: room for n rounded up to a power of two)
hipError_t launch_sort(const double* d_in, double* d_out, uint64_t* d_keys, long n, hipStream_t s);

}  // namespace hbk
