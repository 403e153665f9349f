// hb_mcmc -- command-line front end equivalent to the reference's
//   ./HB_MCMC NITER TIC log10P run          (src/README.txt:7; mcmc_wrapper2.c:70-73)
// with the likelihood on the GPU (libhbmi.so, one batched launch per step).
// The reference's hard-coded root /scratch/ssolanski/HB_MCMC becomes --root
// (default $HB_MCMC_ROOT, else "."); the file tree below it is unchanged:
//   data/lightcurves/folded_lightcurves/<TIC>_new.txt   (input, :254-298)
//   data/magnitudes/<TIC>.txt                           (input, :300-328)
//   data/{chains,logL,log,pars,subpars}, data/lightcurves/mcmc_lightcurves,
//   debug/temp_<j>_log.txt                              (outputs)
// Extra options: --chains W --npast K --ladder 0|1 --threads T --device D --quiet
//   --device-sampler: the whole iteration on the GPU (hb_mcmc_run_device)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../../include/hb_sampler.h"
#include "../../include/hbmi.h"

struct Ctx {
  hb_ctx* ctx;
  long n;
};

static int cb_loglik(void* u, const double* P, int W, double* out) {
  return hb_loglik_batch(((Ctx*)u)->ctx, P, W, out, nullptr);
}
static int cb_model(void* u, const double* P, double* out) {
  return hb_light_curve_batch(((Ctx*)u)->ctx, P, 1, out, nullptr);
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s NITER TIC log10P run [--root DIR] [--chains W] [--npast K] [--ladder 0|1] "
                    "[--threads T] [--device D] [--quiet]\n", argv[0]);
    return 2;
  }
  hb_mcmc_cfg cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.niter = (long)atoi(argv[1]);
  const std::string run_id = argv[2];
  cfg.log10_period = atof(argv[3]);
  cfg.run = atoi(argv[4]);
  cfg.nchains = 50;   // NCHAINS, mcmc_wrapper2.h:11
  cfg.npast = 500;    // NPAST, mcmc_wrapper2.h:12
  cfg.verbose = 1;
  int device = 0;
  bool device_sampler = false;
  const char* envroot = getenv("HB_MCMC_ROOT");
  std::string root = envroot ? envroot : ".";
  for (int i = 5; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--root") root = next();
    else if (a == "--chains") cfg.nchains = atoi(next());
    else if (a == "--npast") cfg.npast = atoi(next());
    else if (a == "--ladder") cfg.ladder = atoi(next());
    else if (a == "--threads") cfg.nthreads = atoi(next());
    else if (a == "--device") device = atoi(next());
    else if (a == "--quiet") cfg.verbose = 0;
    else if (a == "--device-sampler") device_sampler = true;
    else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
  }
  cfg.out_root = root.c_str();
  cfg.run_id = run_id.c_str();
  if (cfg.verbose)
    printf("Using libhbmi (GPU batched likelihood, %s, %d chains)\n",
           device_sampler ? "device-resident sampler" : "host sampler", cfg.nchains);

  const std::string dfname = root + "/data/lightcurves/folded_lightcurves/" + run_id + "_new.txt";
  const std::string magname = root + "/data/magnitudes/" + run_id + ".txt";
  if (cfg.verbose) printf("Opening folded lc data file %s \n", dfname.c_str());
  FILE* fd = fopen(dfname.c_str(), "r");
  if (!fd) {
    printf("Lightcurve datafile not found; terminating program \n");  // :279-283
    return 0;
  }
  long nt = 0;
  if (fscanf(fd, "%ld\n", &nt) != 1 || nt < 2) { fclose(fd); fprintf(stderr, "bad header\n"); return 1; }
  std::vector<double> t(nt), f(nt), e(nt);
  for (long i = 0; i < nt; ++i)
    if (fscanf(fd, "%lf\t%lf\t%lf\n", &t[i], &f[i], &e[i]) != 3) { fclose(fd); fprintf(stderr, "short file\n"); return 1; }
  fclose(fd);
  double mag[5] = {1000., 1., 1., 1., 1.}, magerr[4] = {1.e15, 1.e15, 1.e15, 1.e15};
  FILE* fm = fopen(magname.c_str(), "r");
  if (fm) {  // :302-317
    if (cfg.verbose) printf("Using color / GMAG information \n");
    double a = 0, b = 0;
    if (fscanf(fm, "%lf\n", &a) == 1) mag[0] = a;
    for (int i = 0; i < 4; ++i)
      if (fscanf(fm, "%lf\t%lf\n", &a, &b) == 2) { mag[i + 1] = a; magerr[i] = b; }
    fclose(fm);
  } else if (cfg.verbose) {
    printf("Magnitude file not found/used; assigning infinite error to mag data \n");
  }
  Ctx c;
  c.ctx = hb_create(t.data(), f.data(), e.data(), nt, mag, magerr, device);
  c.n = nt;
  if (!c.ctx) { fprintf(stderr, "hb_create: %s\n", hb_last_error()); return 1; }
  hb_reserve(c.ctx, cfg.nchains);
  hb_mcmc_result res;
  const int rc = device_sampler ? hb_mcmc_run_device(&cfg, c.ctx, t.data(), f.data(), nt, &res)
                                : hb_mcmc_run(&cfg, t.data(), f.data(), e.data(), nt, cb_loglik, cb_model, &c, &res);
  hb_destroy(c.ctx);
  if (rc != 0) { fprintf(stderr, "hb_mcmc_run failed (%d): %s\n", rc, hb_last_error()); return 1; }
  if (cfg.verbose)
    printf("done: %ld iterations, %ld logL evals, %.3f s total, %.3f s in the likelihood; logLmap %.12g\n",
           cfg.niter, res.loglik_evals, res.seconds_total, res.seconds_loglik, res.logLmap);
  return 0;
}
