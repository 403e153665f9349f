/*
 * hbmi.h -- C-ABI of libhbmi.so, the MI355X (gfx950) implementation of the
 * sidruns30/HB_MCMC heartbeat-binary light-curve model and log-likelihood.
 *
 * Part 1 is a drop-in for the reference header `src/likelihood3.h`: the same
 * symbol names, argument types and meanings, so `mcmc_wrapper2.c` (or any
 * other caller of likelihood3.c) links against libhbmi.so unchanged.  Every
 * compute entry point runs on the GPU.  Each prototype cites the reference
 * declaration it replaces (likelihood3.h:line) and its definition
 * (likelihood3.c:line).
 *
 * Part 2 is the batched interface the reference lacks: a context holding one
 * observed light curve resident in HBM and a launch that evaluates W walkers
 * at once (one workgroup per walker).  No torch or HIP types appear in the
 * signatures: streams are passed as `void *` (a hipStream_t, NULL = default).
 *
 * Compile-time configuration mirrored from likelihood3.h:11-29:
 * USE_GMAG=1, USE_COLOR_INFO=0, ALPHA_FREE=ALPHA_MORE=BLENDING=1, NPARS=21.
 */
#ifndef HBMI_H
#define HBMI_H

#ifdef __cplusplus
extern "C" {
#endif

#define HBMI_NPARS 21

/* ---- structs, likelihood3.h:39-66 (identical layout) ---- */
#ifndef HBMI_NO_L3_STRUCTS
struct bounds {
  double lo;
  double hi;
};
struct gauss_bounds {
  int flag;
};
#define HBMI_NTAB 32
struct RNG_Vars {
  long idum2;
  long iy;
  long iv[HBMI_NTAB];
  int iset;
  double gset;
  long cts;
};
typedef struct bounds bounds;
typedef struct gauss_bounds gauss_bounds;
typedef struct RNG_Vars RNG_Vars;
#endif

/* ===================== Part 1: likelihood3.h drop-in ===================== */

/* likelihood3.h:68 / likelihood3.c:48-64.  Lomuto partition of arr[low..high]
 * around arr[high]; returns the pivot's final index (as double, like the
 * reference).  Runs as one device lane (exact Lomuto order). */
double partition(double arr[], int low, int high);

/* likelihood3.h:69 / likelihood3.c:70-83.  Sorts arr[low..high] ascending on
 * the GPU (bitonic sort of order-preserving keys: LDS tiles, then global
 * merge steps).  Output equals quickSort's for all non-NaN inputs; the
 * relative order of -0.0 and +0.0 (which compare equal) may differ. */
void quickSort(double arr[], int low, int high);

/* likelihood3.h:70 / likelihood3.c:86-105.  Subtracts the element of rank
 * n/2 (n even) or n/2+1 (n odd), n = end-begin, from arr[begin..end).
 * Exact radix-select on the GPU.  n < 2 is rejected (arr unchanged; the
 * reference reads out of bounds). */
void remove_median(double *arr, long begin, long end);

/* likelihood3.h:71-72 / likelihood3.c:125-185.  traj_pars = {M1[g], M2[g],
 * P[s], e, inc, omega0, T0[s]}; per time: sky separation d [cm], Z1, Z2 [cm],
 * radial separation rr [cm], true anomaly ff [rad]. */
void traj(double *times, double *traj_pars, double *d_arr, double *Z1_arr, double *Z2_arr,
          double *rr_arr, double *ff_arr, int Nt);

/* likelihood3.h:73 / likelihood3.c:194-209 */
double get_alpha_beam(double logT);
/* likelihood3.h:74-75 / likelihood3.c:224-236 */
double beaming(double P, double M1, double M2, double e, double inc, double omega0, double nu,
               double alpha_beam);
/* likelihood3.h:76-77 / likelihood3.c:255-307 (argument `a` unused, as in the reference) */
double ellipsoidal(double P, double M1, double M2, double e, double inc, double omega0, double nu,
                   double R1, double a, double mu, double tau);
/* likelihood3.h:78-79 / likelihood3.c:322-337 */
double reflection(double P, double M1, double M2, double e, double inc, double omega0, double nu,
                  double R2, double alpha_ref1);
/* likelihood3.h:80 / likelihood3.c:353-389: radii in Rsun, d in cm */
double eclipse_area(double R1, double R2, double d);
/* likelihood3.h:81-82 / likelihood3.c:725-795 */
void calc_mags(double params[], double D, double *Gmg, double *BminusV, double *VminusG,
               double *GminusT);
/* likelihood3.h:83 / likelihood3.c:530-686 */
void calc_light_curve(double *times, long Nt, double *pars, double *template_);
/* likelihood3.h:84 / likelihood3.c:693-717 */
void calc_radii_and_Teffs(double params[], double *R1, double *R2, double *Teff1, double *Teff2);
/* likelihood3.h:85 / likelihood3.c:953-974 */
int RocheOverflow(double *pars);
/* likelihood3.h:86-87 / likelihood3.c:809-873.  Like the reference, clamps
 * noise[i] < 1e-5 to 1e-5 IN THE CALLER'S ARRAY (likelihood3.c:824-827).
 * The light curve stays resident on the GPU between calls with the same
 * contents (per calling thread), so repeated calls only move 21 doubles. */
double loglikelihood(double time[], double lightcurve[], double noise[], long N, double params[],
                     double mag_data[], double magerr[]);
/* likelihood3.h:88 / likelihood3.c:986-1121 (prior box; host-side table) */
void set_limits(bounds limited[], bounds limits[], gauss_bounds gauss_pars[], double LC_PERIOD);
/* likelihood3.h:89 / likelihood3.c:1123-1211 (proposal widths; history untouched) */
void initialize_proposals(double *sigma, double ***history);

/* un-prototyped in likelihood3.h but used by pyHB (likelihood3.pxd:7-13):
 * likelihood3.c:396-438, 445-476, 483-493, 495-507 */
double _getT(double logM);
double _getR(double logM);
double envelope_Temp(double logM);
double envelope_Radius(double logM);
/* likelihood3.c:945-948 */
double Eggleton_RL(double q);
/* likelihood3.c:880-941 (SAVECOMP = 0): the model light curve at 10 000
 * times spanning 30 d + one period, written to `fname` as "%12.5e\t%12.5e"
 * lines (time [d], flux).  The light curve is computed on the GPU. */
void write_lc_to_file(double pars[], char fname[]);

/* ===================== Part 2: batched MI355X interface ===================== */

typedef struct hb_ctx hb_ctx;

/* Upload one observed light curve (t [d], flux, sigma; N cadences) plus the
 * magnitude block {D[pc], G, B-V, V-G, G-T} and its errors (4) to `device`.
 * sigma is clamped to >= 1e-5 in the device copy (the caller's array is not
 * touched).  Returns NULL on error (see hb_last_error); N must be >= 2. */
hb_ctx *hb_create(const double *t, const double *f, const double *sigma, long N,
                  const double *mag_data5, const double *magerr4, int device);
void hb_destroy(hb_ctx *ctx);
long hb_ctx_ncad(const hb_ctx *ctx);

/* Pre-size the per-walker workspace for up to max_walkers (makes the launch
 * entry points allocation-free, hence hipGraph-capturable). 0 on success. */
int hb_reserve(hb_ctx *ctx, int max_walkers);

/* W walkers, params row-major W x 21 (likelihood3.c:533-578 slot order).
 * `_dev` variants take device pointers and are asynchronous on `stream`;
 * the plain variants take host pointers and return after completion.
 * Return 0 on success, negative on error. */
int hb_loglik_batch_dev(hb_ctx *ctx, const double *d_params, int W, double *d_logl, void *stream);
int hb_loglik_batch(hb_ctx *ctx, const double *params, int W, double *logl, void *stream);

/* The two launches behind hb_loglik_batch_dev when it is not fused (below),
 * exposed for timing: hb_prepare_dev computes the per-walker constant records
 * (one lane per walker) into the context workspace; hb_evaluate_dev runs the
 * one-workgroup-per-walker model + median + chi^2 kernel on them (mode 0: logL
 * into d_out[W], mode 1: templates into d_out[W x N]).  Same stream, same W. */
int hb_prepare_dev(hb_ctx *ctx, const double *d_params, int W, void *stream);
int hb_evaluate_dev(hb_ctx *ctx, int W, double *d_out, int mode, void *stream);
/* Walkers per workgroup of the fused launch hb_loglik_batch_dev makes for W
 * walkers (the records computed in the eval kernel's prologue: ONE launch), or
 * 0 when it makes the two launches above.  Fused: one-wave plans of up to 1024
 * cadences, W up to 16 walkers per compute unit (4096 on MI355X).  Either way
 * the records and the phase table the context keeps are the same, and so are
 * the logL values (bit for bit). */
int hb_ctx_fused_wpb(const hb_ctx *ctx, int W);

/* Model light curves (median removed, blended), row-major W x N. */
int hb_light_curve_batch_dev(hb_ctx *ctx, const double *d_params, int W, double *d_out, void *stream);
int hb_light_curve_batch(hb_ctx *ctx, const double *params, int W, double *out, void *stream);

/* Which kernel variant serves this context: waves per walker (1..16) and
 * whether the template lives in LDS (1) or in an HBM scratch slab (0). */
int hb_ctx_waves_per_walker(const hb_ctx *ctx);
int hb_ctx_template_in_lds(const hb_ctx *ctx);
/* Eval kernel the context launches: 0 hb_eval_wave_kernel (lane rows: one wave
 * per walker up to N = 1280, a pair up to 2048, four waves up to 4096; see
 * hb_ctx_waves_per_walker), 1 hb_eval_block_kernel (register keys, N <= 32 x
 * 64 x waves), 2 hb_eval_kernel (LDS-walking select; template in LDS or an
 * HBM slab). */
int hb_ctx_eval_kind(const hb_ctx *ctx);
/* on != 0: batches of fewer than 512 walkers (N <= 2048) run the multi-wave
 * kernel (several waves per walker: lower latency when most SIMDs would sit
 * idle).  Default off: one wave per walker at every batch size, which keeps a
 * context's results bit-identical across batch sizes and with the device
 * sampler (the two kernels sum chi2 in different orders; both within the
 * stated tolerance of likelihood3.c).  Opt-in only (HBLikelihood(latency_plan=
 * True)): the drop-in loglikelihood() keeps the one-wave plan, because the
 * relinked reference sampler is bound by its own host threads (18.6 vs 23.7 us
 * of device time per call, no measurable change in iterations/s;
 * profiles/r02e_latency_probe.txt).  Returns 0. */
int hb_ctx_set_latency_plan(hb_ctx *ctx, int on);

/* Last error message of the calling thread ("" if none). */
const char *hb_last_error(void);

/* ---- catalog mode (config C5): many independent light curves on one GPU.
 * Target k: t[k], flux[k], sigma[k] of n[k] cadences (2..2048), magnitude
 * data mag5[5k..5k+4] / magerr4[4k..4k+3] (NULL: the reference fallback
 * {1000,1,1,1,1} / 1e15).  All light curves are concatenated in HBM with a
 * per-target descriptor table; one call evaluates every target's walkers
 * with one prep launch and ONE eval launch holding every cadences-per-lane
 * class (instead of one small launch per target).  params: sum(walkers[k]) x 21
 * rows, target 0's walkers first, then target 1's, ...; logl likewise. ---- */
typedef struct hb_catalog hb_catalog;
hb_catalog *hb_catalog_create(int ntargets, const double *const *t, const double *const *flux,
                              const double *const *sigma, const long *n, const double *mag5,
                              const double *magerr4, int device);
void hb_catalog_destroy(hb_catalog *cat);
int hb_catalog_ntargets(const hb_catalog *cat);
int hb_catalog_loglik(hb_catalog *cat, const double *params, const int *walkers, double *logl, void *stream);
int hb_catalog_loglik_dev(hb_catalog *cat, const double *d_params, const int *walkers, double *d_logl,
                          void *stream);

/* 1 if a HIP device is usable, 0 otherwise (never falls back to the CPU). */
int hb_device_available(void);

/* ---- measurement helpers (bench.py): HIP events recorded on the caller's
 * stream without the system-scope release fence a default event record
 * performs, so a bracket costs the stream as little as possible. ---- */
void *hb_timer_create(void);
int hb_timer_record(void *timer, void *stream);
float hb_timer_elapsed_ms(void *start, void *stop); /* synchronises on stop; <0 on error */
void hb_timer_destroy(void *timer);

#ifdef __cplusplus
}
#endif
#endif /* HBMI_H */
