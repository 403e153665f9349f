/* ref_batch.c -- OpenMP batch driver around the REFERENCE loglikelihood()
 * (likelihood3.c:809-873, compiled unmodified into _ref/libref_lik3.so).
 * Used as bench.py's cpu_baseline (kind "reference") and by the golden
 * generator.  Test/measurement infrastructure only. */
#include <omp.h>

double loglikelihood(double time[], double lightcurve[], double noise[], long N, double params[],
                     double mag_data[], double magerr[]);

void ref_loglike_batch(double *t, double *f, double *sig, long n, double *pw, long w, double *mag,
                       double *magerr, double *out, int nthreads) {
    /* clamp once so the threads never race on sig[] (the reference clamps
     * inside every call, likelihood3.c:824-827; values are identical) */
    for (long k = 0; k < n; ++k)
        if (sig[k] < 1.e-5) sig[k] = 1.e-5;
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (long j = 0; j < w; ++j) out[j] = loglikelihood(t, f, sig, n, pw + 21 * j, mag, magerr);
}
