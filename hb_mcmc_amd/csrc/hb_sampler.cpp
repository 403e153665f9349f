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

#include "../../include/hb_sampler.h"
#include "../../include/hbmi.h"

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
void apply_walls(double* y, const Prior& pr) {
  for (int i = 0; i < kNp; ++i) {
    const double lo = pr.limits[i].lo, hi = pr.limits[i].hi;
    for (long guard = 0; guard < 100000000L; ++guard) {
      const bool below = (pr.limited[i].lo == 1) && (y[i] < lo);
      const bool above = (pr.limited[i].hi == 1) && (y[i] > hi);
      if (!(below || above)) break;
      y[i] = (y[i] < lo) ? 2.0 * lo - y[i] : 2.0 * hi - y[i];
    }
    for (long guard = 0; (pr.limited[i].lo == 2) && (y[i] < lo) && guard < 100000000L; ++guard)
      y[i] = hi + (y[i] - lo);
    for (long guard = 0; (pr.limited[i].hi == 2) && (y[i] > hi) && guard < 100000000L; ++guard)
      y[i] = lo + (y[i] - hi);
  }
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

extern "C" int hb_mcmc_run(const hb_mcmc_cfg* cfg, const double* t, const double* fl_data, const double* sigma,
                           long n, hb_loglik_fn loglik, hb_model_fn model, void* user, hb_mcmc_result* res) {
  if (!cfg || !loglik || cfg->nchains < 2 || cfg->npast < 2 || n < 2) return -1;
  const int W = cfg->nchains, NPAST = cfg->npast;
  const long NITER = cfg->niter;
  if (cfg->ladder == 0 && W > 2000) return -2;  // 1.4^i overflows: the reference would hang
  int nth = cfg->nthreads;
  if (nth <= 0) {
    const unsigned hw = std::thread::hardware_concurrency();
    nth = hw == 0 ? 1 : (int)(hw > 16 ? 16 : hw);
  }
  Pool pool(nth);
  std::mutex log_mu;
  const double log_lc_period = cfg->log10_period;
  const double LC_PERIOD = pow(10., log_lc_period);
  srand((unsigned)NITER);  // :86

  std::vector<long> seeds(W);
  std::vector<RNG_Vars> states(W);
  for (int i = 0; i < W; ++i) {  // :88-106
    seeds[i] = i + cfg->run;
    memset(&states[i], 0, sizeof(RNG_Vars));
    states[i].idum2 = 123456789;
  }
  Prior pr;
  set_limits(pr.limited, pr.limits, pr.gp, LC_PERIOD);  // :195
  double sigma_p[kNp];
  initialize_proposals(sigma_p, nullptr);  // :198

  // random initial state from chain 0's stream (USE_RAND_PARS=1, :233-252)
  std::vector<double> x((size_t)W * kNp), xmap(kNp);
  for (int i = 0; i < kNp; ++i)
    for (int j = 0; j < W; ++j) {
      const double u = ran2p(&seeds[0], &states[0]);
      double v = pr.limits[i].lo + u * (pr.limits[i].hi - pr.limits[i].lo);
      if (i == 2) v = log_lc_period;
      if (i == 6) v = fmod(v, LC_PERIOD);
      x[(size_t)j * kNp + i] = v;
    }

  std::vector<double> temp(W);
  std::vector<int> index(W);
  const double dtemp = 1.4;  // :331-339
  temp[0] = 1.0;
  index[0] = 0;
  for (int i = 1; i < W; ++i) {
    temp[i] = (cfg->ladder == 1 && i % 50 == 0) ? 1.0 : temp[i - 1] * dtemp;
    index[i] = i;
  }

  double t_loglik = 0.;
  long n_evals = 0;
  auto eval = [&](const double* P, int w, double* out) -> int {
    const double t0 = now_s();
    const int rc = loglik(user, P, w, out);
    t_loglik += now_s() - t0;
    n_evals += w;
    return rc;
  };

  std::vector<double> logLx(W), logPx(W);
  double logLmap;
  if (eval(x.data(), 1, &logLmap)) return -3;  // :342 (chain 0's state)
  for (int i = 0; i < W; ++i) logLx[i] = logLmap;
  for (int i = 0; i < kNp; ++i) xmap[i] = x[i];  // xmap is uninitialised in the reference; only printed after updates
  if (cfg->verbose) printf("initial chi2 and likelihood %lf \t %lf\n", -2 * logLmap, logLmap);

  Files files;
  if (cfg->out_root && cfg->out_root[0]) {
    if (!open_files(files, cfg->out_root, cfg->run_id ? cfg->run_id : "run", cfg->run, W)) return -4;
  }
  std::vector<double> model_buf(model ? n : 0);

  // history[j][k][:] (NPAST x 21 per temperature slot)
  std::vector<double> hist((size_t)W * NPAST * kNp, 0.0);
  std::vector<const double*> hrow((size_t)W * NPAST);
  for (size_t r = 0; r < hrow.size(); ++r) hrow[r] = &hist[r * kNp];

  std::vector<int> acc_arr(W, 0), DEacc_arr(W, 0), DEtrial_arr(W, 0);
  std::vector<double> y((size_t)W * kNp), logLy(W), logPy(W), alpha2(W), xcur((size_t)W * kNp);
  std::vector<int> jump(W), jtype(W);
  long acc = 0, DEacc = 0, DEtrial = 0, atrial = 0;
  long cold_acc = 0, nswap = 0;
  const double t_start = now_s();

  for (long iter = 0; iter < NITER; ++iter) {
    const int k = (int)(iter - (iter / NPAST) * NPAST);
    // ---- proposals (:386-485), one RNG stream per temperature slot j ----
    pool.run(W, [&](int j) {
      RNG_Vars* st = &states[j];
      long* sd = &seeds[j];
      const int chain_id = index[j];
      const double* xc = &x[(size_t)chain_id * kNp];
      double* yj = &y[(size_t)j * kNp];
      const double a = ran2p(sd, st);
      const double jscale = pow(10., -6. + 6. * a);
      int jmp = 0, jt = 0;
      if ((ran2p(sd, st) < 0.5) && (iter > NPAST)) jmp = 1;
      if (jmp == 0) {
        gaussian_step(xc, sd, sigma_p, jscale, temp[j], yj, st);
        jt = 1;
      }
      if (jmp == 1) {
        if (chain_id == 0) DEtrial_arr[j]++;
        de_step(xc, sd, &hrow[(size_t)j * NPAST], NPAST, yj, st);
        jt = 2;
        double dx_mag = 0;
        for (int i = 0; i < kNp; ++i) dx_mag += (xc[i] - yj[i]) * (xc[i] - yj[i]);
        if (dx_mag < 1e-6) {
          gaussian_step(xc, sd, sigma_p, jscale, temp[j], yj, st);
          jt = 1;
        }
      }
      apply_walls(yj, pr);
      if (yj[1] > yj[0]) {  // "order the masses" (:470-475): y[1] = y[0], as written
        const double keep = yj[1];
        (void)keep;
        yj[1] = yj[0];
        yj[0] = yj[1];
      }
      yj[2] = log_lc_period;
      yj[6] = fmod(yj[6], LC_PERIOD);
      logPx[chain_id] = log_prior(xc, pr);
      logPy[j] = log_prior(yj, pr);
      jump[j] = jmp;
      jtype[j] = jt;
      alpha2[j] = ran2p(sd, st);  // drawn after the likelihood calls in the reference; same stream order
    });
    // ---- likelihoods: one batch (two at iteration 0) ----
    if (iter == 0) {
      for (int j = 0; j < W; ++j)
        memcpy(&xcur[(size_t)j * kNp], &x[(size_t)index[j] * kNp], sizeof(double) * kNp);
      std::vector<double> lx(W);
      if (eval(xcur.data(), W, lx.data())) return -3;
      for (int j = 0; j < W; ++j) logLx[index[j]] = lx[j];
    }
    if (eval(y.data(), W, logLy.data())) return -3;
    // ---- Hastings test and history (:492-546) ----
    pool.run(W, [&](int j) {
      const int chain_id = index[j];
      double* xc = &x[(size_t)chain_id * kNp];
      const double* yj = &y[(size_t)j * kNp];
      const double H = exp((logLy[j] - logLx[chain_id]) / temp[j] + (logPy[j] - logPx[chain_id]));
      if (alpha2[j] <= H) {
        if ((logLx[chain_id] / logLy[j] <= 0.5) && (iter > 10000) && (j <= 5) && files.on) {
          std::lock_guard<std::mutex> lk(log_mu);
          log_big_jump(files.log, iter, chain_id, H, alpha2[j], temp[j], logLx[chain_id], logLy[j],
                       logPx[chain_id], logPy[j], xc, yj, jtype[j]);
        }
        if (chain_id == 0) acc_arr[j]++;
        memcpy(xc, yj, sizeof(double) * kNp);
        logLx[chain_id] = logLy[j];
        if ((jump[j] == 1) && (chain_id == 0)) DEacc_arr[j]++;
      }
      memcpy(&hist[((size_t)j * NPAST + k) * kNp], xc, sizeof(double) * kNp);
    });
    // ---- statistics and tempering swaps (:554-563) ----
    for (int i = 0; i < W; ++i) {
      acc += acc_arr[i];
      cold_acc += acc_arr[i];
      DEacc += DEacc_arr[i];
      DEtrial += DEtrial_arr[i];
      acc_arr[i] = 0;
      // ptmcmc (:768-817)
      const int b = (int)(((double)rand() / (RAND_MAX)) * ((double)(W - 1)));
      const int a = b + 1;
      const int olda = index[a], oldb = index[b];
      const double heat1 = temp[a], heat2 = temp[b];
      const double dlogL = logLx[oldb] - logLx[olda];
      const double Hs = (heat2 - heat1) / (heat2 * heat1);
      const double al = exp(dlogL * Hs);
      const double be = ((double)rand() / (RAND_MAX));
      if (al >= be) {
        index[a] = oldb;
        index[b] = olda;
        ++nswap;
      }
    }
    if (logLx[index[0]] > logLmap) {  // :565-572
      memcpy(xmap.data(), &x[(size_t)index[0] * kNp], sizeof(double) * kNp);
      logLmap = logLx[index[0]];
    }
    if (cfg->verbose && iter % 1000 == 0) {  // :575-589
      printf("%ld/%ld logL=%.10g acc=%.3g DEacc=%.3g", iter, NITER, logLx[index[0]], (double)(acc) / ((double)atrial),
             (double)DEacc / (double)DEtrial);
      printf("\n");
      printf("Parameter values: \n");
      for (int i = 0; i < 5; ++i) printf("%lf\t", x[(size_t)index[W > 10 ? 10 : W - 1] * kNp + i]);
      printf("\n");
    }
    atrial++;
    if ((iter % 100 == 0) && files.on) {  // :593-649
      fprintf(files.chain, "%ld %.12g ", iter / 10, logLx[index[0]]);
      for (int i = 0; i < kNp; ++i) fprintf(files.chain, "%.12g ", x[(size_t)index[0] * kNp + i]);
      fprintf(files.chain, "\n");
      fprintf(files.logl, "%ld ", iter / 10);
      for (int i = 0; i < W; ++i) {
        fprintf(files.logl, "%.12g ", logLx[index[i]]);
        for (int jj = 0; jj < kNp; ++jj) fprintf(files.temps[i], "%lf\t", x[(size_t)index[i] * kNp + jj]);
        fprintf(files.temps[i], "\n");
      }
      fprintf(files.logl, "\n");
      acc = atrial = 0;
      for (int i = 0; i < W; ++i) DEtrial_arr[i] = DEacc_arr[i] = acc_arr[i] = 0;
      if (model) {
        if (model(user, xmap.data(), model_buf.data())) return -5;
        write_lc(files, t, fl_data, model_buf.data(), n);
      }
      write_pars(files.subparname, &x[(size_t)index[0] * kNp]);
    }
  }
  if (files.on) {  // :655-681
    if (model) {
      if (model(user, xmap.data(), model_buf.data())) return -5;
      write_lc(files, t, fl_data, model_buf.data(), n);
    }
    write_pars(files.parname, &x[(size_t)index[0] * kNp]);
    fclose(files.log);
    fclose(files.chain);
    fclose(files.logl);
    for (FILE* f : files.temps) fclose(f);
    if (files.swap) fclose(files.swap);
  }
  (void)sigma;
  if (res) {
    memcpy(res->xmap, xmap.data(), sizeof(double) * kNp);
    res->logLmap = logLmap;
    res->accepted = cold_acc;
    res->swaps = nswap;
    res->seconds_total = now_s() - t_start;
    res->seconds_loglik = t_loglik;
    res->loglik_evals = n_evals;
  }
  return 0;
}
