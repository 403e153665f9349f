// hb_sampler.cpp -- parallel-tempered Metropolis-Hastings caller of the HB
// likelihood, equivalent to sidruns30/HB_MCMC src/mcmc_wrapper2.c (main loop
// :378-650, helpers :703-1178), with the per-chain likelihood calls of
// :488-489 replaced by ONE batched call per step:
//   * iteration 0 evaluates every chain's current state (the reference's
//     recompute at :488 only differs from the stored value at iteration 0,
//     where logLx[] holds logL(x[0]) for every chain, :342-347);
//   * every iteration evaluates all proposals y at once.
// Host work per step (proposals, reflecting/periodic walls, priors, Hastings,
// history) runs OpenMP-parallel over chains; every chain owns its RNG stream,
// so results do not depend on the thread count.  The tempering swaps (:554-563)
// stay sequential on glibc rand(), seeded with srand(NITER) (:86).
// Parallel loops use a small persistent std::thread pool (no OpenMP runtime
// in libhbmi.so, so it coexists with torch's and numpy's).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <chrono>
#include <string>
#include <vector>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <memory>
#include <utility>

#include "../../include/hb_sampler.h"
#include "../../include/hbmi.h"
#include "hb_lagfib.hpp"
#include "hb_sampler_view.hpp"
#include "hb_walls.hpp"

namespace {

constexpr int kNp = HBMI_NPARS;
constexpr double kSqrt2Pi = 2.5066282746;  // mcmc_wrapper2.h:10
constexpr double kBigNum = 1.e15;          // likelihood3.h:31

// --------------------------------------------------------------------------
// L'Ecuyer generator with Bays-Durham shuffle, per chain (:894-943).  Only a
// non-positive seed initialises the table (:905); the reference seeds chain i
// with i + run (:91), so only chain 0 of run 0 shuffles -- reproduced as is.
// --------------------------------------------------------------------------
constexpr long IM1 = 2147483563, IM2 = 2147483399, IMM1 = IM1 - 1;
constexpr long IA1 = 40014, IA2 = 40692, IQ1 = 53668, IQ2 = 52774, IR1 = 12211, IR2 = 3791;
constexpr int NTAB = HBMI_NTAB;
constexpr long NDIV = 1 + IMM1 / NTAB;
constexpr double AM = 1.0 / IM1;
constexpr double RNMX = 1.0 - 1.2e-7;

double ran2p(long* idum, RNG_Vars* st) {
  st->cts += 1;
  if (*idum <= 0) {
    *idum = (-(*idum) < 1) ? 1 : -(*idum);
    st->idum2 = *idum;
    for (int j = NTAB + 7; j >= 0; --j) {
      const long k = *idum / IQ1;
      *idum = IA1 * (*idum - k * IQ1) - k * IR1;
      if (*idum < 0) *idum += IM1;
      if (j < NTAB) st->iv[j] = *idum;
    }
    st->iy = st->iv[0];
  }
  long k = *idum / IQ1;
  *idum = IA1 * (*idum - k * IQ1) - k * IR1;
  if (*idum < 0) *idum += IM1;
  k = st->idum2 / IQ2;
  st->idum2 = IA2 * (st->idum2 - k * IQ2) - k * IR2;
  if (st->idum2 < 0) st->idum2 += IM2;
  const int j = (int)(st->iy / NDIV);
  st->iy = st->iv[j] - st->idum2;
  st->iv[j] = *idum;
  if (st->iy < 1) st->iy += IMM1;
  const double temp = AM * st->iy;
  return temp > RNMX ? RNMX : temp;
}

// Marsaglia polar Gaussian, cached second deviate per chain (:947-974)
double gasdevp(long* idum, RNG_Vars* st) {
  if (*idum < 0) st->iset = 0;
  if (st->iset == 0) {
    double v1, v2, rsq;
    do {
      v1 = 2.0 * ran2p(idum, st) - 1.0;
      v2 = 2.0 * ran2p(idum, st) - 1.0;
      rsq = v1 * v1 + v2 * v2;
    } while (rsq >= 1.0 || rsq == 0.0);
    const double fac = sqrt(-2.0 * log(rsq) / rsq);
    st->gset = v1 * fac;
    st->iset = 1;
    return v2 * fac;
  }
  st->iset = 0;
  return st->gset;
}

double gauss_pdf(double x, double mean, double sigma) {  // :1175-1178
  return (1 / sigma / kSqrt2Pi) * exp(-pow((x - mean) / sigma, 2.) / 2.);
}

struct Prior {
  bounds limited[kNp], limits[kNp];
  gauss_bounds gp[kNp];
};

// get_logP (:703-765): Gaussian priors on the flagged slots
double log_prior(const double* x, const Prior& pr) {
  double lp = 0.;
  for (int i = 0; i < kNp; ++i) {
    double mean, sig;
    if (i == 7 || i == 8) { mean = 0.; sig = 1.; }
    else if (i == 9 || i == 11) { mean = 0.16; sig = 0.04; }
    else if (i == 10 || i == 12) { mean = 0.34; sig = 0.04; }
    else if (i == 13 || i == 14) { mean = 1.; sig = 0.2; }
    else if (i == 15 || i == 16) { mean = 0.; sig = 0.1; }
    else if (i == 17 || i == 18) { mean = 0.; sig = 1.; }
    else { mean = 0.; sig = kBigNum; }
    if (pr.gp[i].flag == 1) lp += log(gauss_pdf(x[i], mean, sig));
  }
  return lp;
}

// reflecting (flag 1) and periodic (flag 2) walls (:440-467).  The reference
// loops forever on a non-finite coordinate; here such a coordinate is left
// alone after a bounded number of folds (it yields NaN logL -> rejection).
// Long reflection runs (hot chains) are fast-forwarded exactly (hb_walls.hpp).
void apply_walls(double* y, const Prior& pr) {
  for (int i = 0; i < kNp; ++i)
    y[i] = hbwall::apply_wall(y[i], pr.limits[i].lo, pr.limits[i].hi, pr.limited[i].lo, pr.limited[i].hi);
}

void gaussian_step(const double* x, long* seed, const double* sigma, double scale, double temp, double* y,
                   RNG_Vars* st) {  // :1062-1088
  const double sqtemp = sqrt(temp);
  double dx[kNp];
  for (int n = 0; n < kNp; ++n) dx[n] = gasdevp(seed, st) * sigma[n] * sqtemp * scale;
  for (int n = 0; n < kNp; ++n) y[n] = x[n] + dx[n];
}

// differential evolution (:1091-1140) as compiled: `a` is overwritten by a
// second draw truncated to 0 (:1103-1104); the uninitialised `c` of
// gaussian(c, 0, 1e-4) (:1099, :1115) is what gcc -O3 materialises, 0
// (`xor %ecx,%ecx`), so epsilon = dx * (gaussian(0, 0, 1e-4) - 0.5).
void de_step(const double* x, long* seed, const double* const* hist, int npast, double* y, RNG_Vars* st) {
  int a = (int)(ran2p(seed, st) * npast);
  a = (int)ran2p(seed, st);
  int b = a;
  while (b == a) b = (int)(ran2p(seed, st) * npast);
  const int c = 0;
  double dx[kNp], eps[kNp];
  for (int n = 0; n < kNp; ++n) {
    dx[n] = hist[b][n] - hist[a][n];
    eps[n] = dx[n] * (gauss_pdf(c, 0, 1.e-4) - 0.5);
  }
  if (ran2p(seed, st) < 0.9) {
    const double gamma = 2.388 / sqrt(2. * kNp);  // GAMMA, mcmc_wrapper2.h:13
    for (int n = 0; n < kNp; ++n) dx[n] *= gasdevp(seed, st) * gamma;
  }
  for (int n = 0; n < kNp; ++n) {
    dx[n] += eps[n];
    y[n] = x[n] + dx[n];
  }
}

// glibc's rand() (random_r TYPE_3: r[k] = r[k-31] + r[k-3] mod 2^32, output
// r[k] >> 1, seeded by srandom_r's Schrage recurrence and 310 discarded
// outputs), held per sampler.  The reference calls the process-global
// rand() after srand(NITER) (:86, :778-812); a private copy of the same
// sequence cannot be perturbed by a library (RCCL's lazy communicator setup,
// say) that calls rand() in between.  Checked against libc by test_sampler.py.
class GlibcRand {
 public:
  explicit GlibcRand(unsigned seed = 1) { srand(seed); }
  void srand(unsigned seed) {
    if (seed == 0) seed = 1;
    int32_t word = (int32_t)seed;
    r_[0] = (uint32_t)word;
    for (int i = 1; i < 31; ++i) {
      const int32_t hi = word / 127773, lo = word % 127773;
      word = 16807 * lo - 2836 * hi;
      if (word < 0) word += 2147483647;
      r_[i] = (uint32_t)word;
    }
    for (int i = 31; i < 34; ++i) r_[i] = r_[i - 31];
    k_ = 34;
    for (int i = 0; i < 310; ++i) next();
  }
  int rand() { return (int)(next() >> 1); }
  // the last 31 outputs r[k-31 .. k-1] (the generator's whole state)
  void window(uint32_t* w) const {
    for (int i = 0; i < 31; ++i) w[i] = r_[(k_ - 31 + i) % 34];
  }
  // skip n outputs (hb_lagfib.hpp jump-ahead; the device sampler's schedule
  // producers consume the stream from a copy)
  void skip(unsigned long long n) {
    if (n == 0) return;
    uint32_t w[31], c[31];
    window(w);
    hblf::poly_xpow(n, c);
    hblf::window_jump(w, c);
    k_ += (long)n;
    for (int i = 0; i < 31; ++i) r_[(k_ - 31 + i) % 34] = w[i];
  }

 private:
  uint32_t next() {  // ring of 34: r[k-31] = r[(k+3) % 34], r[k-3] = r[(k+31) % 34]
    const uint32_t v = r_[(k_ + 3) % 34] + r_[(k_ + 31) % 34];
    r_[k_ % 34] = v;
    ++k_;
    return v;
  }
  uint32_t r_[34];
  long k_ = 0;
};

struct Files {
  FILE* chain = nullptr;
  FILE* logl = nullptr;
  FILE* log = nullptr;
  FILE* swap = nullptr;
  std::vector<FILE*> temps;
  std::string outname, subparname, parname;
  bool on = false;
};

void mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); ++i) {
    cur += path[i];
    if (path[i] == '/' && cur.size() > 1) mkdir(cur.c_str(), 0755);
  }
  mkdir(path.c_str(), 0755);
}

// file layout of mcmc_wrapper2.c:110-173 and :360-374 under `root`
bool open_files(Files& fl, const char* root, const char* run_id, int run, int nchains) {
  const std::string r(root);
  const std::string suffix = std::string(run_id) + "_gmag" + "_OMP" + "_" + std::to_string(run);
  for (const char* d : {"/data/subpars", "/data/pars", "/data/chains", "/data/logL", "/data/log",
                        "/data/lightcurves/mcmc_lightcurves", "/debug"})
    mkdirs(r + d);
  fl.subparname = r + "/data/subpars/subpar." + suffix + ".dat";
  fl.parname = r + "/data/pars/par." + suffix + ".dat";
  fl.outname = r + "/data/lightcurves/mcmc_lightcurves/" + suffix + ".out";
  fl.chain = fopen((r + "/data/chains/chain." + suffix + ".dat").c_str(), "w");
  fl.logl = fopen((r + "/data/logL/logL." + suffix + ".dat").c_str(), "w");
  fl.log = fopen((r + "/data/log/log." + suffix + ".dat").c_str(), "w");
  if (!fl.chain || !fl.logl || !fl.log) return false;
  fl.temps.resize(nchains, nullptr);
  for (int j = 0; j < nchains; ++j) {
    const std::string tn = r + "/debug/temp_" + std::to_string(j) + "_log.txt";
    fl.temps[j] = fopen(tn.c_str(), "w");
    if (!fl.temps[j]) return false;
  }
  fl.swap = fopen((r + "/debug/temp_swap_file.txt").c_str(), "w");  // opened, never written (:374)
  fl.on = true;
  return true;
}

void write_lc(const Files& fl, const double* t, const double* f, const double* m, long n) {
  FILE* fh = fopen(fl.outname.c_str(), "w");
  if (!fh) return;
  fprintf(fh, "%ld\n", n);
  for (long i = 0; i < n; ++i) fprintf(fh, "%12.5e %12.5e %12.5e\n", t[i], f[i], m[i]);
  fclose(fh);
}

void write_pars(const std::string& name, const double* x) {
  FILE* fh = fopen(name.c_str(), "w");
  if (!fh) return;
  for (int z = 0; z < kNp; ++z) fprintf(fh, "%12.5e ", x[z]);
  fprintf(fh, "\n");
  fclose(fh);
}

void log_big_jump(FILE* lf, long iter, int chain_id, double H, double alpha, double tmp, double lx, double ly,
                  double px, double py, const double* xo, const double* xn, int jump_type) {  // :1230-1255
  fprintf(lf, "Big jump in likelihood detected on iternation: %ld and chain id: %ld ;", iter, (long)chain_id);
  fprintf(lf, " temperature of the chain: %f \n", tmp);
  fprintf(lf, "Old log prior: %f new log prior: %f old log likelihood: %f new log likelihood: %f \n", px, py, lx, ly);
  fprintf(lf, "Hastings ratio [exp((logLy-logLx[chain_id])/temp[j]) * pow(10., logPy - logPx)] %f, alpha %f \
          and jump type %d\n", H, alpha, jump_type);
  fprintf(lf, "Printing old and new parameters \n");
  for (int i = 0; i < kNp; ++i) fprintf(lf, "%lf \t", xo[i]);
  fprintf(lf, "\n");
  for (int i = 0; i < kNp; ++i) fprintf(lf, "%lf \t", xn[i]);
  fprintf(lf, "\n ************************************************ \n");
}

// fixed-partition parallel-for over [0, n): chunk c = [c*n/T, (c+1)*n/T)
class Pool {
 public:
  explicit Pool(int nthreads) : T_(nthreads < 1 ? 1 : nthreads) {
    for (int i = 1; i < T_; ++i) th_.emplace_back([this, i] { worker(i); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(int n, const std::function<void(int)>& body) {
    if (T_ == 1 || n < 2 * T_) {
      for (int i = 0; i < n; ++i) body(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      body_ = &body;
      n_ = n;
      pending_ = T_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    chunk(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
  }

 private:
  void chunk(int c) {
    const int lo = (int)((long)n_ * c / T_), hi = (int)((long)n_ * (c + 1) / T_);
    for (int i = lo; i < hi; ++i) (*body_)(i);
  }
  void worker(int c) {
    long seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      chunk(c);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  int T_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* body_ = nullptr;
  int n_ = 0, pending_ = 0;
  long gen_ = 0;
  bool stop_ = false;
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" double hb_ran2_parallel(long* idum, void* st) { return ran2p(idum, (RNG_Vars*)st); }
extern "C" double hb_gasdev2_parallel(long* idum, void* st) { return gasdevp(idum, (RNG_Vars*)st); }
extern "C" int hb_rand_stream(unsigned seed, int n, int* out) {
  GlibcRand g(seed);
  for (int i = 0; i < n; ++i) out[i] = g.rand();
  return 0;
}

// the same stream after jumping `skip` draws ahead (hb_lagfib.hpp)
extern "C" int hb_rand_stream_jump(unsigned seed, unsigned long long skip, int n, int* out) {
  GlibcRand g(seed);
  g.skip(skip);
  for (int i = 0; i < n; ++i) out[i] = g.rand();
  return 0;
}

// ---------------------------------------------------------------------------
// Output files of mcmc_wrapper2.c (:110-173, :593-681), fed by slot.
// ---------------------------------------------------------------------------
struct hb_writer {
  Files files;
  int W = 0;
  std::mutex mu;  // big-jump log lines come from the Hastings worker threads
};

extern "C" hb_writer* hb_writer_open(const char* root, const char* run_id, int run, int W) {
  if (!root || !root[0] || W < 1) return nullptr;
  hb_writer* w = new hb_writer();
  w->W = W;
  if (!open_files(w->files, root, run_id ? run_id : "run", run, W)) {
    delete w;
    return nullptr;
  }
  return w;
}

// iteration block of :593-649 (chain / logL / per-temperature logs); x_slots
// and logl_slots are the post-swap states by temperature slot (slot 0 = cold)
extern "C" int hb_writer_step(hb_writer* w, long iter, const double* logl_slots, const double* x_slots) {
  if (!w) return -1;
  Files& fl = w->files;
  fprintf(fl.chain, "%ld %.12g ", iter / 10, logl_slots[0]);
  for (int i = 0; i < kNp; ++i) fprintf(fl.chain, "%.12g ", x_slots[i]);
  fprintf(fl.chain, "\n");
  fprintf(fl.logl, "%ld ", iter / 10);
  for (int i = 0; i < w->W; ++i) {
    fprintf(fl.logl, "%.12g ", logl_slots[i]);
    for (int jj = 0; jj < kNp; ++jj) fprintf(fl.temps[i], "%lf\t", x_slots[(size_t)i * kNp + jj]);
    fprintf(fl.temps[i], "\n");
  }
  fprintf(fl.logl, "\n");
  return 0;
}

extern "C" int hb_writer_lc(hb_writer* w, const double* t, const double* f, const double* m, long n) {
  if (!w) return -1;
  write_lc(w->files, t, f, m, n);
  return 0;
}

// which = 0: subpar (every 100 iterations), 1: final par file
extern "C" int hb_writer_pars(hb_writer* w, int which, const double* x) {
  if (!w) return -1;
  write_pars(which ? w->files.parname : w->files.subparname, x);
  return 0;
}

extern "C" void hb_writer_close(hb_writer* w) {
  if (!w) return;
  Files& fl = w->files;
  fclose(fl.log);
  fclose(fl.chain);
  fclose(fl.logl);
  for (FILE* f : fl.temps) fclose(f);
  if (fl.swap) fclose(fl.swap);
  delete w;
}

// ---------------------------------------------------------------------------
// The sampler state, owned by temperature SLOT.  The reference keeps chain
// states by chain id and permutes index[] on a swap (:768-817); here slot j
// holds the state of the chain currently at temperature j (plus that chain's
// id and logL), so a contiguous slot range [lo, hi) can live on one rank and
// a swap only moves the two chains' 21-double records.  With lo = 0, hi = W
// this is exactly the single-process sampler.
// ---------------------------------------------------------------------------
constexpr int kRec = kNp + 2;  // x[21], logL, chain id

struct hb_sampler {
  int W = 0, NPAST = 0, lo = 0, hi = 0, nl = 0;
  long NITER = 0;
  double log_lc_period = 0, LC_PERIOD = 0;
  Prior pr;
  double sigma_p[kNp];
  std::vector<double> temp;                    // W (the whole ladder)
  std::vector<long> seeds;                     // nl
  std::vector<RNG_Vars> states;                // nl
  std::vector<double> x, logL, logP;           // nl x 21, nl, nl
  std::vector<char> logP_ok;                   // logP[jl] == log_prior(x[jl]) (cache; the state is unchanged)
  std::vector<int> cid;                        // nl: chain id at the slot
  std::vector<double> y, logPy, alpha2;        // proposals
  std::vector<int> jump, jtype;
  std::vector<double> hist;                    // nl x NPAST x 21
  std::vector<const double*> hrow;
  std::vector<int> acc_arr, DEacc_arr, DEtrial_arr;
  long acc = 0, DEacc = 0, DEtrial = 0, atrial = 0, cold_acc = 0, nswap = 0;
  GlibcRand rng;                                // the swap draws (srand(NITER), :86)
  std::vector<int> perm;                        // W, scratch of swap()
  std::vector<double> Lperm;                    // W
  std::vector<double> old, oldP;                // nl x kRec, nl: scratch of apply_perm()
  std::vector<char> oldP_ok;
  hb_writer* log = nullptr;
  Pool* pool = nullptr;
  ~hb_sampler() { delete pool; }
};

extern "C" hb_sampler* hb_sampler_create(const hb_mcmc_cfg* cfg, int slot_lo, int slot_hi) {
  if (!cfg || cfg->nchains < 2 || cfg->npast < 2) return nullptr;
  const int W = cfg->nchains;
  if (cfg->ladder == 0 && W > 2000) return nullptr;  // 1.4^i overflows: the reference would hang
  if (slot_lo < 0 || slot_hi > W || slot_lo >= slot_hi) return nullptr;
  hb_sampler* s = new hb_sampler();
  s->W = W;
  s->NPAST = cfg->npast;
  s->NITER = cfg->niter;
  s->lo = slot_lo;
  s->hi = slot_hi;
  s->nl = slot_hi - slot_lo;
  int nth = cfg->nthreads;
  if (nth <= 0) {
    const unsigned hw = std::thread::hardware_concurrency();
    nth = hw == 0 ? 1 : (int)(hw > 16 ? 16 : hw);
  }
  s->pool = new Pool(nth);
  s->log_lc_period = cfg->log10_period;
  s->LC_PERIOD = pow(10., s->log_lc_period);
  s->rng.srand((unsigned)s->NITER);  // :86 (every rank replays the same swap draws)
  const int nl = s->nl;

  // chain 0's stream draws the initial states of ALL chains (USE_RAND_PARS=1,
  // :233-252); every rank replays it and keeps its own slots
  RNG_Vars st0;
  memset(&st0, 0, sizeof st0);
  st0.idum2 = 123456789;
  long seed0 = 0 + cfg->run;
  set_limits(s->pr.limited, s->pr.limits, s->pr.gp, s->LC_PERIOD);  // :195
  initialize_proposals(s->sigma_p, nullptr);                           // :198
  s->x.resize((size_t)nl * kNp);
  for (int i = 0; i < kNp; ++i)
    for (int j = 0; j < W; ++j) {
      const double u = ran2p(&seed0, &st0);
      double v = s->pr.limits[i].lo + u * (s->pr.limits[i].hi - s->pr.limits[i].lo);
      if (i == 2) v = s->log_lc_period;
      if (i == 6) v = fmod(v, s->LC_PERIOD);
      if (j >= slot_lo && j < slot_hi) s->x[(size_t)(j - slot_lo) * kNp + i] = v;
    }
  s->seeds.resize(nl);
  s->states.resize(nl);
  for (int jl = 0; jl < nl; ++jl) {  // :88-106
    s->seeds[jl] = slot_lo + jl + cfg->run;
    memset(&s->states[jl], 0, sizeof(RNG_Vars));
    s->states[jl].idum2 = 123456789;
  }
  if (slot_lo == 0) {  // chain 0 continues its stream after the initial draws
    s->seeds[0] = seed0;
    s->states[0] = st0;
  }

  s->temp.resize(W);
  s->temp[0] = 1.0;  // :331-339
  for (int i = 1; i < W; ++i) s->temp[i] = (cfg->ladder == 1 && i % 50 == 0) ? 1.0 : s->temp[i - 1] * 1.4;

  s->logL.assign(nl, 0.0);
  s->logP.assign(nl, 0.0);
  s->logP_ok.assign(nl, 0);
  s->cid.resize(nl);
  for (int jl = 0; jl < nl; ++jl) s->cid[jl] = slot_lo + jl;
  s->y.resize((size_t)nl * kNp);
  s->logPy.resize(nl);
  s->alpha2.resize(nl);
  s->jump.resize(nl);
  s->jtype.resize(nl);
  s->hist.assign((size_t)nl * s->NPAST * kNp, 0.0);
  s->hrow.resize((size_t)nl * s->NPAST);
  for (size_t r = 0; r < s->hrow.size(); ++r) s->hrow[r] = &s->hist[r * kNp];
  s->acc_arr.assign(nl, 0);
  s->DEacc_arr.assign(nl, 0);
  s->DEtrial_arr.assign(nl, 0);
  s->perm.resize(W);
  s->Lperm.resize(W);
  s->old.resize((size_t)nl * kRec);
  return s;
}

extern "C" void hb_sampler_destroy(hb_sampler* s) { delete s; }

extern "C" int hb_sampler_attach_log(hb_sampler* s, hb_writer* w) {
  if (!s) return -1;
  s->log = w;
  return 0;
}

// current states / logL / chain ids of the owned slots
extern "C" int hb_sampler_get(const hb_sampler* s, double* x_out, double* logl_out, int* cid_out) {
  if (!s) return -1;
  if (x_out) memcpy(x_out, s->x.data(), sizeof(double) * s->x.size());
  if (logl_out) memcpy(logl_out, s->logL.data(), sizeof(double) * s->nl);
  if (cid_out) memcpy(cid_out, s->cid.data(), sizeof(int) * s->nl);
  return 0;
}

// logL of the current states (the reference's recompute at :488, which only
// changes anything at iteration 0)
extern "C" int hb_sampler_set_logl(hb_sampler* s, const double* logl) {
  if (!s || !logl) return -1;
  memcpy(s->logL.data(), logl, sizeof(double) * s->nl);
  return 0;
}

// proposals of the owned slots (:386-485); y_out: nl x 21
extern "C" int hb_sampler_propose(hb_sampler* s, long iter, double* y_out) {
  if (!s) return -1;
  const int NPAST = s->NPAST, lo = s->lo;
  s->pool->run(s->nl, [&](int jl) {
    RNG_Vars* st = &s->states[jl];
    long* sd = &s->seeds[jl];
    const int j = lo + jl;
    const int chain_id = s->cid[jl];
    const double* xc = &s->x[(size_t)jl * kNp];
    double* yj = &s->y[(size_t)jl * kNp];
    const double a = ran2p(sd, st);
    const double jscale = pow(10., -6. + 6. * a);
    int jmp = 0, jt = 0;
    if ((ran2p(sd, st) < 0.5) && (iter > NPAST)) jmp = 1;
    if (jmp == 0) {
      gaussian_step(xc, sd, s->sigma_p, jscale, s->temp[j], yj, st);
      jt = 1;
    }
    if (jmp == 1) {
      if (chain_id == 0) s->DEtrial_arr[jl]++;
      de_step(xc, sd, &s->hrow[(size_t)jl * NPAST], NPAST, yj, st);
      jt = 2;
      double dx_mag = 0;
      for (int i = 0; i < kNp; ++i) dx_mag += (xc[i] - yj[i]) * (xc[i] - yj[i]);
      if (dx_mag < 1e-6) {
        gaussian_step(xc, sd, s->sigma_p, jscale, s->temp[j], yj, st);
        jt = 1;
      }
    }
    apply_walls(yj, s->pr);
    if (yj[1] > yj[0]) {  // "order the masses" (:470-475): y[1] = y[0], as written
      yj[1] = yj[0];
      yj[0] = yj[1];
    }
    yj[2] = s->log_lc_period;
    yj[6] = fmod(yj[6], s->LC_PERIOD);
    if (!s->logP_ok[jl]) {  // :444 recomputes it every step; the value only changes with the state
      s->logP[jl] = log_prior(xc, s->pr);
      s->logP_ok[jl] = 1;
    }
    s->logPy[jl] = log_prior(yj, s->pr);
    s->jump[jl] = jmp;
    s->jtype[jl] = jt;
    s->alpha2[jl] = ran2p(sd, st);  // drawn after the likelihood calls in the reference; same stream order
  });
  if (y_out) memcpy(y_out, s->y.data(), sizeof(double) * s->y.size());
  return 0;
}

// Hastings test and history (:492-546) for the owned slots; logly: nl
extern "C" int hb_sampler_accept(hb_sampler* s, long iter, const double* logly) {
  if (!s || !logly) return -1;
  const int NPAST = s->NPAST, lo = s->lo;
  const int k = (int)(iter - (iter / NPAST) * NPAST);
  s->pool->run(s->nl, [&](int jl) {
    const int j = lo + jl;
    const int chain_id = s->cid[jl];
    double* xc = &s->x[(size_t)jl * kNp];
    const double* yj = &s->y[(size_t)jl * kNp];
    const double H = exp((logly[jl] - s->logL[jl]) / s->temp[j] + (s->logPy[jl] - s->logP[jl]));
    if (s->alpha2[jl] <= H) {
      if ((s->logL[jl] / logly[jl] <= 0.5) && (iter > 10000) && (j <= 5) && s->log) {
        std::lock_guard<std::mutex> lk(s->log->mu);
        log_big_jump(s->log->files.log, iter, chain_id, H, s->alpha2[jl], s->temp[j], s->logL[jl], logly[jl],
                     s->logP[jl], s->logPy[jl], xc, yj, s->jtype[jl]);
      }
      if (chain_id == 0) s->acc_arr[jl]++;
      memcpy(xc, yj, sizeof(double) * kNp);
      s->logL[jl] = logly[jl];
      s->logP[jl] = s->logPy[jl];  // log_prior(y), computed in propose
      if ((s->jump[jl] == 1) && (chain_id == 0)) s->DEacc_arr[jl]++;
    }
    memcpy(&s->hist[((size_t)jl * NPAST + k) * kNp], xc, sizeof(double) * kNp);
  });
  // statistics of the swap loop (:554-558): acc_arr is cleared every step,
  // the DE counters only every 100 steps (:640), so DEacc/DEtrial add up
  // running totals -- reproduced as written
  for (int jl = 0; jl < s->nl; ++jl) {
    s->acc += s->acc_arr[jl];
    s->cold_acc += s->acc_arr[jl];
    s->DEacc += s->DEacc_arr[jl];
    s->DEtrial += s->DEtrial_arr[jl];
    s->acc_arr[jl] = 0;
  }
  return 0;
}

// Tempering swaps (ptmcmc, :768-817), W sequential attempts on glibc rand().
// logl_all: logL by slot for ALL W slots; every rank replays the same draws
// on the same values and so reaches the same permutation.  perm_out[j] = the
// slot whose chain sits at slot j afterwards; logl_perm_out (optional) the
// permuted logL.  Returns the number of accepted swaps.
extern "C" int hb_sampler_swap(hb_sampler* s, const double* logl_all, int* perm_out, double* logl_perm_out) {
  if (!s || !logl_all) return -1;
  const int W = s->W;
  int* p = s->perm.data();
  double* L = s->Lperm.data();
  for (int j = 0; j < W; ++j) {
    p[j] = j;
    L[j] = logl_all[j];
  }
  int n = 0;
  for (int i = 0; i < W; ++i) {
    const int b = (int)(((double)s->rng.rand() / (RAND_MAX)) * ((double)(W - 1)));
    const int a = b + 1;
    const double be = ((double)s->rng.rand() / (RAND_MAX));
    // rand() == RAND_MAX gives b = W-1: the reference then reads index[NCHAINS]
    // out of bounds (:791-797); here that attempt is void (draws consumed)
    if (a >= W) continue;
    const double heat1 = s->temp[a], heat2 = s->temp[b];
    const double dlogL = L[b] - L[a];
    const double Hs = (heat2 - heat1) / (heat2 * heat1);
    const double al = exp(dlogL * Hs);
    if (al >= be) {
      std::swap(p[a], p[b]);
      std::swap(L[a], L[b]);
      ++n;
    }
  }
  s->nswap += n;
  if (perm_out) memcpy(perm_out, p, sizeof(int) * W);
  if (logl_perm_out) memcpy(logl_perm_out, L, sizeof(double) * W);
  return n;
}

// record {x[21], logL, chain id} of an owned slot
extern "C" int hb_sampler_pack(const hb_sampler* s, int slot, double* rec) {
  if (!s || slot < s->lo || slot >= s->hi) return -1;
  const int jl = slot - s->lo;
  memcpy(rec, &s->x[(size_t)jl * kNp], sizeof(double) * kNp);
  rec[kNp] = s->logL[jl];
  rec[kNp + 1] = (double)s->cid[jl];
  return 0;
}

// Moves the chains to their slots after swap(): owned slot j takes the chain
// of slot perm[j]; when that slot is owned by another rank its record comes
// from remote[(j - lo) * 23 ...] (filled by the caller's exchange).
extern "C" int hb_sampler_apply_perm(hb_sampler* s, const int* perm, const double* remote) {
  if (!s || !perm) return -1;
  const int nl = s->nl, lo = s->lo, hi = s->hi;
  for (int jl = 0; jl < nl; ++jl) hb_sampler_pack(s, lo + jl, &s->old[(size_t)jl * kRec]);
  s->oldP.assign(s->logP.begin(), s->logP.end());
  s->oldP_ok.assign(s->logP_ok.begin(), s->logP_ok.end());
  for (int jl = 0; jl < nl; ++jl) {
    const int src = perm[lo + jl];
    const double* r;
    if (src >= lo && src < hi) {
      r = &s->old[(size_t)(src - lo) * kRec];
      s->logP[jl] = s->oldP[src - lo];
      s->logP_ok[jl] = s->oldP_ok[src - lo];
    } else {
      if (!remote) return -2;
      r = &remote[(size_t)jl * kRec];
      s->logP_ok[jl] = 0;  // recomputed from the received state
    }
    memcpy(&s->x[(size_t)jl * kNp], r, sizeof(double) * kNp);
    s->logL[jl] = r[kNp];
    s->cid[jl] = (int)r[kNp + 1];
  }
  return 0;
}

// running statistics of the owned slots: {acc, DEacc, DEtrial, atrial,
// cold_acc, nswap}; end_iter() does :590 and the 100-step reset of :639-641
extern "C" int hb_sampler_stats(const hb_sampler* s, long* out6) {
  if (!s || !out6) return -1;
  out6[0] = s->acc;
  out6[1] = s->DEacc;
  out6[2] = s->DEtrial;
  out6[3] = s->atrial;
  out6[4] = s->cold_acc;
  out6[5] = s->nswap;
  return 0;
}

extern "C" int hb_sampler_export(const hb_sampler* s, long* seeds, void* states, double* hist) {
  if (!s) return -1;
  if (seeds) memcpy(seeds, s->seeds.data(), sizeof(long) * s->nl);
  if (states) memcpy(states, s->states.data(), sizeof(RNG_Vars) * s->nl);
  if (hist) memcpy(hist, s->hist.data(), sizeof(double) * s->hist.size());
  return 0;
}

extern "C" int hb_sampler_end_iter(hb_sampler* s, long iter) {
  if (!s) return -1;
  s->atrial++;
  if (iter % 100 == 0) {
    s->acc = s->atrial = 0;
    for (int jl = 0; jl < s->nl; ++jl) s->DEtrial_arr[jl] = s->DEacc_arr[jl] = s->acc_arr[jl] = 0;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Internal bridge for the device-resident sampler (hb_dsampler.hip).
// ---------------------------------------------------------------------------
extern "C" int hbx_sampler_view(hb_sampler* s, HbSamplerView* v) {
  if (!s || !v) return -1;
  v->W = s->W;
  v->NPAST = s->NPAST;
  v->lo = s->lo;
  v->hi = s->hi;
  v->nl = s->nl;
  v->NITER = s->NITER;
  v->log_lc_period = s->log_lc_period;
  v->LC_PERIOD = s->LC_PERIOD;
  v->limited = s->pr.limited;
  v->limits = s->pr.limits;
  v->gp = s->pr.gp;
  v->sigma_p = s->sigma_p;
  v->temp = s->temp.data();
  v->seeds = s->seeds.data();
  v->states = s->states.data();
  v->x = s->x.data();
  v->logL = s->logL.data();
  v->logP = s->logP.data();
  v->logP_ok = s->logP_ok.data();
  v->cid = s->cid.data();
  v->hist = s->hist.data();
  v->acc_arr = s->acc_arr.data();
  v->DEacc_arr = s->DEacc_arr.data();
  v->DEtrial_arr = s->DEtrial_arr.data();
  v->acc = &s->acc;
  v->DEacc = &s->DEacc;
  v->DEtrial = &s->DEtrial;
  v->atrial = &s->atrial;
  v->cold_acc = &s->cold_acc;
  v->nswap = &s->nswap;
  v->log = s->log;
  return 0;
}

// the swap stream's state (hb_lagfib.hpp window) and a jump of n draws
extern "C" int hbx_swap_rng_window(const hb_sampler* s, uint32_t* w31) {
  if (!s || !w31) return -1;
  s->rng.window(w31);
  return 0;
}
extern "C" int hbx_swap_rng_skip(hb_sampler* s, unsigned long long n) {
  if (!s) return -1;
  s->rng.skip(n);
  return 0;
}

extern "C" int hbx_swap_draws(hb_sampler* s, int* b, double* beta) {
  if (!s) return -1;
  const int W = s->W;
  for (int i = 0; i < W; ++i) {  // same expressions as hb_sampler_swap / ptmcmc :791, :810
    b[i] = (int)(((double)s->rng.rand() / (RAND_MAX)) * ((double)(W - 1)));
    beta[i] = ((double)s->rng.rand() / (RAND_MAX));
  }
  return 0;
}

extern "C" void hbx_log_big_jump(hb_writer* w, long iter, int chain_id, double H, double alpha, double tmp,
                                 double lx, double ly, double px, double py, const double* xo, const double* xn,
                                 int jump_type) {
  if (!w) return;
  std::lock_guard<std::mutex> lk(w->mu);
  log_big_jump(w->files.log, iter, chain_id, H, alpha, tmp, lx, ly, px, py, xo, xn, jump_type);
}

// ---------------------------------------------------------------------------
// Single-process driver (all W slots local): the mcmc_wrapper2.c main loop.
// ---------------------------------------------------------------------------
extern "C" int hb_mcmc_run(const hb_mcmc_cfg* cfg, const double* t, const double* fl_data, const double* sigma,
                           long n, hb_loglik_fn loglik, hb_model_fn model, void* user, hb_mcmc_result* res) {
  if (!cfg || !loglik || cfg->nchains < 2 || cfg->npast < 2 || n < 2) return -1;
  if (cfg->ladder == 0 && cfg->nchains > 2000) return -2;
  const int W = cfg->nchains;
  const long NITER = cfg->niter;
  std::unique_ptr<hb_sampler, void (*)(hb_sampler*)> sp(hb_sampler_create(cfg, 0, W), hb_sampler_destroy);
  if (!sp) return -1;
  hb_sampler* s = sp.get();

  double t_loglik = 0.;
  long n_evals = 0;
  auto eval = [&](const double* P, int w, double* out) -> int {
    const double t0 = now_s();
    const int rc = loglik(user, P, w, out);
    t_loglik += now_s() - t0;
    n_evals += w;
    return rc;
  };

  std::vector<double> xmap(kNp);
  double logLmap;
  if (eval(s->x.data(), 1, &logLmap)) return -3;  // :342 (chain 0's state)
  memcpy(xmap.data(), s->x.data(), sizeof(double) * kNp);  // uninitialised in the reference; only printed after updates
  if (cfg->verbose) printf("initial chi2 and likelihood %lf \t %lf\n", -2 * logLmap, logLmap);

  std::unique_ptr<hb_writer, void (*)(hb_writer*)> wr(nullptr, hb_writer_close);
  if (cfg->out_root && cfg->out_root[0]) {
    wr.reset(hb_writer_open(cfg->out_root, cfg->run_id, cfg->run, W));
    if (!wr) return -4;
    hb_sampler_attach_log(s, wr.get());
  }
  std::vector<double> model_buf(model ? n : 0), logly(W), lx(W);
  const double t_start = now_s();

  for (long iter = 0; iter < NITER; ++iter) {
    hb_sampler_propose(s, iter, nullptr);
    if (iter == 0) {  // every chain's current state (see header)
      if (eval(s->x.data(), W, lx.data())) return -3;
      hb_sampler_set_logl(s, lx.data());
    }
    if (eval(s->y.data(), W, logly.data())) return -3;
    hb_sampler_accept(s, iter, logly.data());
    hb_sampler_swap(s, s->logL.data(), nullptr, nullptr);
    hb_sampler_apply_perm(s, s->perm.data(), nullptr);
    if (s->logL[0] > logLmap) {  // :565-572
      memcpy(xmap.data(), s->x.data(), sizeof(double) * kNp);
      logLmap = s->logL[0];
    }
    if (cfg->verbose && iter % 1000 == 0) {  // :575-589
      printf("%ld/%ld logL=%.10g acc=%.3g DEacc=%.3g", iter, NITER, s->logL[0], (double)(s->acc) / ((double)s->atrial),
             (double)s->DEacc / (double)s->DEtrial);
      printf("\n");
      printf("Parameter values: \n");
      for (int i = 0; i < 5; ++i) printf("%lf\t", s->x[(size_t)(W > 10 ? 10 : W - 1) * kNp + i]);
      printf("\n");
    }
    if ((iter % 100 == 0) && wr) {  // :593-649
      hb_writer_step(wr.get(), iter, s->logL.data(), s->x.data());
      if (model) {
        if (model(user, xmap.data(), model_buf.data())) return -5;
        hb_writer_lc(wr.get(), t, fl_data, model_buf.data(), n);
      }
      hb_writer_pars(wr.get(), 0, s->x.data());
    }
    hb_sampler_end_iter(s, iter);
  }
  if (wr) {  // :655-681
    if (model) {
      if (model(user, xmap.data(), model_buf.data())) return -5;
      hb_writer_lc(wr.get(), t, fl_data, model_buf.data(), n);
    }
    hb_writer_pars(wr.get(), 1, s->x.data());
  }
  (void)sigma;
  if (res) {
    memcpy(res->xmap, xmap.data(), sizeof(double) * kNp);
    res->logLmap = logLmap;
    res->accepted = s->cold_acc;
    res->swaps = s->nswap;
    res->seconds_total = now_s() - t_start;
    res->seconds_loglik = t_loglik;
    res->loglik_evals = n_evals;
  }
  return 0;
}
