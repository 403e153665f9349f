/*
 * hb_oracle.c -- CPU restatement of the heartbeat-binary (HB) light-curve
 * model and chi^2 log-likelihood of sidruns30/HB_MCMC `src/likelihood3.c`.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity *checker*: only
 * `tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of
 * `bench.py` may load it.  The product path (hb_mcmc_amd/, libhbmi.so) never
 * links, calls or falls back to it.
 *
 * Every routine restates one reference routine with the SAME floating-point
 * operation order (left-associative products, the same temporaries, the same
 * libm calls) so that, built with `gcc -O3 -ffp-contract=off` against the
 * same glibc libm, it is bit-identical to the reference compiled the way its
 * README prescribes (`gcc -O3 -std=c99`, x86-64 baseline ISA => no FMA).
 * That claim is pinned by tests/test_oracle_golden.py against vectors the
 * reference itself produced (tests/golden/make_golden.py).
 *
 * Reference map (file:line in /root/reference/src):
 *   orc_median_shift      <- remove_median/quickSort/partition  likelihood3.c:36-105
 *   orc_orbit             <- traj                                likelihood3.c:125-185
 *   orc_beam_coeff        <- get_alpha_beam                      likelihood3.c:194-209
 *   orc_doppler           <- beaming                             likelihood3.c:224-236
 *   orc_tidal             <- ellipsoidal                         likelihood3.c:255-307
 *   orc_irradiation       <- reflection                          likelihood3.c:322-337
 *   orc_overlap           <- eclipse_area                        likelihood3.c:353-389
 *   orc_logteff_table     <- _getT                               likelihood3.c:396-438
 *   orc_logrstar_table    <- _getR                               likelihood3.c:445-476
 *   orc_teff_spread       <- envelope_Temp                       likelihood3.c:483-493
 *   orc_radius_spread     <- envelope_Radius                     likelihood3.c:495-507
 *   orc_light_curve       <- calc_light_curve                    likelihood3.c:530-686
 *   orc_stellar           <- calc_radii_and_Teffs                likelihood3.c:693-717
 *   orc_photometry        <- calc_mags                           likelihood3.c:725-795
 *   orc_loglike           <- loglikelihood                       likelihood3.c:809-873
 *   orc_write_lc_file     <- write_lc_to_file                    likelihood3.c:880-941
 *   orc_lobe_fraction     <- Eggleton_RL                         likelihood3.c:945-948
 *   orc_roche_flag        <- RocheOverflow                       likelihood3.c:953-974
 * Compile-time configuration mirrored: USE_GMAG=1, USE_COLOR_INFO=0,
 * ALPHA_FREE=ALPHA_MORE=BLENDING=1 => 21 parameters (likelihood3.h:11-29).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* physical constants, likelihood3.h:4-10, 31 */
#define K_PI 3.14159265358979323846
#define K_GRAV 6.6743e-8
#define K_CLIGHT 2.998e10
#define K_MSUN 1.9885e33
#define K_RSUN 6.955e10
#define K_DAY 86400.0
#define K_HUGE 1.e15

/* ------------------------------------------------------------------ */
/* median removal: Lomuto quicksort, last element as pivot              */
/* ------------------------------------------------------------------ */
static void orc_exch(double *u, double *v)
{
    double keep = *u;
    *u = *v;
    *v = keep;
}

/* Lomuto partition (likelihood3.c:48-64).  Returned as double, like the
 * reference prototype. */
double orc_partition(double *v, int lo, int hi)
{
    double piv = v[hi];
    int slot = lo - 1;
    for (int k = lo; k < hi; ++k) {
        if (v[k] < piv) {
            ++slot;
            orc_exch(&v[slot], &v[k]);
        }
    }
    orc_exch(&v[slot + 1], &v[hi]);
    return (double)(slot + 1);
}

void orc_quicksort(double *v, int lo, int hi)
{
    if (lo < hi) {
        int p = (int)orc_partition(v, lo, hi);
        orc_quicksort(v, lo, p - 1);
        orc_quicksort(v, p + 1, hi);
    }
}

/* remove_median (likelihood3.c:86-105): the subtracted element is
 * sorted[n/2] for even n and sorted[n/2+1] for odd n (one above the true
 * median; n == 1 reads past the end in the reference -- callers must not). */
void orc_median_shift(double *v, long first, long last)
{
    long n = last - first;
    double *tmp = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    for (int k = 0; k < n; ++k) tmp[k] = v[first + k];
    orc_quicksort(tmp, 0, (int)n - 1);
    int pick = (n % 2 == 0) ? (int)(n / 2) : (int)(n / 2) + 1;
    double med = tmp[pick];
    for (int k = 0; k < n; ++k) v[first + k] -= med;
    free(tmp);
}

/* value the reference would subtract (test helper; no mutation) */
double orc_median_value(const double *v, long n)
{
    double *tmp = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    memcpy(tmp, v, (size_t)n * sizeof(double));
    orc_quicksort(tmp, 0, (int)n - 1);
    int pick = (n % 2 == 0) ? (int)(n / 2) : (int)(n / 2) + 1;
    double med = tmp[pick];
    free(tmp);
    return med;
}

/* ------------------------------------------------------------------ */
/* orbit: Kepler solve with 5 Newton steps (likelihood3.c:125-185)       */
/* op[] = {M1 [g], M2 [g], P [s], e, inc, omega0, T0 [s]}                */
/* ------------------------------------------------------------------ */
void orc_orbit(const double *tt, const double *op, double *sep_sky,
               double *z1, double *z2, double *rad, double *anom, int n)
{
    double mA = op[0], mB = op[1], per = op[2], ecc = op[3];
    double incl = op[4], argp = op[5], tperi = op[6];
    if (mB > mA) orc_exch(&mA, &mB);
    double msum = mA + mB;
    double axis = pow(K_GRAV * msum * (per * per) / ((2 * K_PI) * (2 * K_PI)), 1. / 3.);

    for (int k = 0; k < n; ++k) {
        double ts = tt[k] * K_DAY;
        double mean_an = 2. * K_PI * (ts - tperi) / per;
        mean_an = fmod(mean_an, 2 * K_PI);
        double ecc_an = mean_an;
        double sm = sin(mean_an);
        if (sm != 0.0) ecc_an = mean_an + 0.85 * ecc * sm / fabs(sm);
        for (int it = 0; it < 5; ++it)
            ecc_an = ecc_an - (ecc_an - ecc * sin(ecc_an) - mean_an) / (1 - ecc * cos(ecc_an));

        rad[k] = axis * (1 - ecc * cos(ecc_an));
        anom[k] = 2. * atan(sqrt((1. + ecc) / (1. - ecc)) * tan(ecc_an / 2.));

        double cu = cos(argp + anom[k]);
        double su = sin(argp + anom[k]);
        double ci = cos(incl);
        double si = sin(incl);
        double zz = rad[k] * su * si;
        double proj = sqrt((cu * cu) + ((su * ci) * (su * ci)));
        sep_sky[k] = rad[k] * proj;
        z1[k] = zz * (mB / msum);
        z2[k] = -zz * (mA / msum);
    }
}

/* The Kepler solve of orc_orbit alone, from the mean anomaly: start      */
/* M + 0.85 e sign(sin M), five Newton steps (likelihood3.c:152-160).     */
void orc_kepler(const double *mean, long n, double ecc, double *out)
{
    for (long k = 0; k < n; ++k) {
        double mean_an = mean[k];
        double ecc_an = mean_an;
        double sm = sin(mean_an);
        if (sm != 0.0) ecc_an = mean_an + 0.85 * ecc * sm / fabs(sm);
        for (int it = 0; it < 5; ++it)
            ecc_an = ecc_an - (ecc_an - ecc * sin(ecc_an) - mean_an) / (1 - ecc * cos(ecc_an));
        out[k] = ecc_an;
    }
}

/* ------------------------------------------------------------------ */
/* Doppler beaming coefficient table, Claret et al. 2020 (l3.c:194-209)  */
/* ------------------------------------------------------------------ */
double orc_beam_coeff(double lt)
{
    static const double av[4] = {6.5, 4.0, 2.5, 1.2};
    static const double lv[4] = {3.5, 3.7, 3.9, 4.5};
    if (lt >= lv[3]) return 1.2 / 4;
    if (lt < lv[0]) return 6.5 / 4;
    int k = 3;
    while (lt < lv[k]) k--;
    return ((av[k + 1] + (av[k + 1] - av[k]) / (lv[k + 1] - lv[k]) * (lt - lv[k + 1])) / 4);
}

/* beaming (likelihood3.c:224-236).  NB: pow(1+q, 2/3) is integer 2/3 == 0,
 * so the mass-ratio factor is q / 1.0 -- reproduced on purpose. */
double orc_doppler(double pd, double ma, double mb, double ecc, double incl,
                   double argp, double nu, double ab)
{
    double q = mb / ma;
    double f1 = q / pow(1 + q, 0);
    double f2 = pow(ma, 1. / 3);
    double f3 = pow(pd, -1. / 3);
    double f4 = sin(incl) * cos(argp + nu) / sqrt(1 - (ecc * ecc));
    return -2830. * ab * f1 * f2 * f3 * f4 * 1.e-6;
}

/* ellipsoidal variation, Engel et al. 2020 (likelihood3.c:255-307) */
double orc_tidal(double pd, double ma, double mb, double ecc, double incl,
                 double argp, double nu, double rs, double axis, double mu, double tau)
{
    (void)axis; /* unused by the reference as well */
    double a11 = 15 * mu * (2 + tau) / (32 * (3 - mu));
    double a21 = 3 * (15 + mu) * (1 + tau) / (20 * (3 - mu));
    double a2b = 15 * (1 - mu) * (3 + tau) / (64 * (3 - mu));
    double a01 = a21 / 9;
    double a0b = 3 * a2b / 20;
    double a31 = 5 * a11 / 3;
    double a41 = 7 * a2b / 4;

    double bfac = (1 + ecc * cos(nu)) / (1 - (ecc * ecc));
    double q = mb / ma;
    double prot = pd * pow(1 - ecc, 3. / 2);
    double si = sin(incl);
    double s2 = si * si;
    double s3 = (si * si) * si;
    double s4 = ((si * si) * si) * si;
    double br = bfac * rs;
    double br3 = (br * br) * br;
    double br4 = ((br * br) * br) * br;
    double u = argp + nu;

    double t_am1 = 26870 * a01 * (2 - 3 * s2) * (1 / ma) * (1 / (prot * prot)) * ((rs * rs) * rs);
    double t_am2 = 40305 * a01 * (2 - 3 * s2) * (1 / ma) * q / (1 + q) * (1 / (pd * pd)) * br3;
    double t_c21 = 13435 * a21 * s2 * (1 / ma) * q / (1 + q) * (1 / (pd * pd)) * br3 * cos(2 * u);
    double acc = 0.;
    acc += (t_am1 + t_am2 + t_c21) * 1.e-6;

    double t_am3 = 759 * a0b * (8 - 40 * s2 + 35 * s4) * pow(ma, -5. / 3) * q / pow(1 + q, 5. / 3)
                   * pow(pd, -10. / 3) * pow(br, 5);
    double t_s1 = 3194 * a11 * (4 * si - 5 * s3) * pow(ma, -4. / 3) * q / pow(1 + q, 4. / 3)
                  * pow(pd, -8. / 3) * br4 * sin(u);
    double t_c22 = 759 * a2b * (6 * s2 - 7 * s4) * pow(ma, -5. / 3) * q / pow(1 + q, 5. / 3)
                   * pow(pd, -10. / 3) * br * br4 * cos(2 * u);
    double t_s3 = 3194 * a31 * s3 * pow(ma, -4. / 3) * q / pow(1 + q, 4. / 3) * pow(pd, -8. / 3)
                  * br4 * sin(3 * u);
    double t_c4 = 759 * a41 * s4 * pow(ma, -5. / 3) * q / pow(1 + q, 5. / 3) * pow(pd, -10. / 3)
                  * br * br4 * cos(4 * u);
    acc += (t_am3 + t_s1 + t_c22 + t_s3 + t_c4) * 1.e-6;
    return acc;
}

/* reflection, Faigler & Mazeh 2015 via Engel (likelihood3.c:322-337) */
double orc_irradiation(double pd, double ma, double mb, double ecc, double incl,
                       double argp, double nu, double rcomp, double aref)
{
    double q = mb / ma;
    double bfac = (1 + ecc * cos(nu)) / (1 - (ecc * ecc));
    double f1 = pow(1 + q, -2. / 3);
    double f2 = pow(ma, -2. / 3);
    double f3 = pow(pd, -4. / 3);
    double f4 = (bfac * rcomp) * (bfac * rcomp);
    double si = sin(incl);
    double u = argp + nu;
    double f5 = 0.64 - si * sin(u) + 0.18 * (si * si) * (1 - cos(2 * u));
    return 56514 * aref * f1 * f2 * f3 * f4 * f5 * 1.e-6;
}

/* circle-circle overlap (likelihood3.c:353-389); d in cm, radii in Rsun */
double orc_overlap(double ra, double rb, double d)
{
    if (rb > ra) {
        double keep = ra;
        ra = rb;
        rb = keep;
    }
    double area = 0.;
    d = fabs(d) / K_RSUN;
    double dc = sqrt(ra * ra - rb * rb);
    if (d >= (ra + rb)) area = 0.;
    if (d < (ra - rb)) area = K_PI * rb * rb;
    if ((d > dc) & (d < (ra + rb))) {
        double cq = d * d - rb * rb + ra * ra;
        double hh = sqrt((4. * d * d * ra * ra - (cq * cq)) / (4. * d * d));
        double la = ra * ra * asin(hh / ra) - hh * sqrt(ra * ra - hh * hh);
        double lb = rb * rb * asin(hh / rb) - hh * sqrt(rb * rb - hh * hh);
        area = la + lb;
    }
    if ((d <= dc) & (d >= (ra - rb))) {
        double cq = d * d - rb * rb + ra * ra;
        double hh = sqrt((4. * d * d * ra * ra - (cq * cq)) / (4. * d * d));
        double la = ra * ra * asin(hh / ra) - hh * sqrt(ra * ra - hh * hh);
        double lb = rb * rb * asin(hh / rb) - hh * sqrt(rb * rb - hh * hh);
        area = K_PI * rb * rb - (-la + lb);
    }
    return area;
}

/* ------------------------------------------------------------------ */
/* stellar tables (likelihood3.c:396-507)                               */
/* ------------------------------------------------------------------ */
double orc_logteff_table(double lm)
{
    static const double mn[16] = {0.1, 0.26, 0.47, 0.59, 0.69, 0.87, 0.98, 1.085,
                                  1.4, 1.65, 2.0, 2.5, 3.0, 4.4, 15., 40.};
    static const double tn[16] = {3.491, 3.531, 3.547, 3.584, 3.644, 3.712, 3.745, 3.774,
                                  3.823, 3.863, 3.913, 3.991, 4.057, 4.182, 4.477, 4.623};
    double m = pow(10., lm);
    double out = 0.;
    if (m <= mn[0]) return tn[0];
    if (m >= mn[15]) return tn[15];
    for (int k = 0; k < 16; ++k) {
        if (m < mn[k]) {
            out = tn[k - 1] + (m - mn[k - 1]) * (tn[k] - tn[k - 1]) / (mn[k] - mn[k - 1]);
            break;
        }
    }
    return out;
}

double orc_logrstar_table(double lm)
{
    static const double mn[10] = {0.07, 0.2, 0.356, 0.655, 0.784, 0.787, 1.377, 4.4, 15., 40.};
    static const double rn[10] = {-0.953, -0.627, -0.423, -0.154, -0.082, -0.087,
                                  0.295, 0.477, 0.792, 1.041};
    double m = pow(10., lm);
    if (m <= mn[0]) return rn[0];
    if (m >= mn[9]) return rn[9];
    for (int k = 0; k < 10; ++k)
        if (m < mn[k]) return rn[k - 1] + (m - mn[k - 1]) * (rn[k] - rn[k - 1]) / (mn[k] - mn[k - 1]);
    return NAN; /* NaN mass: the reference falls off the end (UB) */
}

double orc_teff_spread(double lm)
{
    (void)lm;
    return 0.0224;
}

double orc_radius_spread(double lm)
{
    double m = pow(10., lm);
    const double ex = 4.22, sl = 15.68, lo = 0.01, knee = 1.055, hi = 0.17;
    return 1 / (1 / hi + 1 / (sl * pow((pow(m, ex) + pow(knee, ex)), (1 / ex)) - (sl * knee - lo)));
}

/* calc_radii_and_Teffs (likelihood3.c:693-717): R in Rsun, T in K */
void orc_stellar(const double *p, double *r1, double *r2, double *t1, double *t2)
{
    *r1 = pow(10., orc_logrstar_table(p[0]) + p[7] * orc_radius_spread(p[0]));
    *r2 = pow(10., orc_logrstar_table(p[1]) + p[8] * orc_radius_spread(p[1]));
    *t1 = pow(10., orc_logteff_table(p[0]) + p[17] * orc_teff_spread(p[0]));
    *t2 = pow(10., orc_logteff_table(p[1]) + p[18] * orc_teff_spread(p[1]));
}

/* ------------------------------------------------------------------ */
/* full light curve (likelihood3.c:530-686)                             */
/* ------------------------------------------------------------------ */
void orc_light_curve(const double *tt, long n, const double *p, double *out)
{
    double per_s = pow(10., p[2]) * K_DAY;
    double per_d = pow(10., p[2]);
    double ecc = p[3], incl = p[4], argp = p[5], tperi = p[6];
    double mu1 = p[9], tau1 = p[10], mu2 = p[11], tau2 = p[12];
    double ref1 = p[13], ref2 = p[14];
    double xb1 = exp(p[15]);
    double xb2 = exp(p[16]);
    double blend = p[19], tune = p[20];

    double m1 = pow(10., p[0]);
    double m2 = pow(10., p[1]);
    double op[7] = {m1 * K_MSUN, m2 * K_MSUN, per_s, ecc, incl, argp, tperi * K_DAY};

    double r1 = 0., r2 = 0., t1 = 0., t2 = 0.;
    orc_stellar(p, &r1, &r2, &t1, &t2);

    double l1 = (r1 * r1) * (((t1 * t1) * t1) * t1);
    double l2 = (r2 * r2) * (((t2 * t2) * t2) * t2);
    double w1 = l1 / (l1 + l2);
    double w2 = l2 / (l1 + l2);

    double ab1 = orc_beam_coeff(log10(t1)) * xb1;
    double ab2 = orc_beam_coeff(log10(t2)) * xb2;

    double mtot = (m1 + m2) * K_MSUN;
    double axis = pow(K_GRAV * mtot * per_s * per_s / (4.0 * K_PI * K_PI), 1. / 3.);
    double axis_rs = axis / K_RSUN;

    double *work = (double *)malloc((size_t)(5 * (n > 0 ? n : 1)) * sizeof(double));
    double *sep = work, *z1 = work + n, *z2 = work + 2 * n, *rad = work + 3 * n, *nu = work + 4 * n;
    orc_orbit(tt, op, sep, z1, z2, rad, nu, (int)n);

    for (int k = 0; k < n; ++k) {
        double b1 = orc_doppler(per_d, m1, m2, ecc, incl, argp, nu[k], ab1);
        double e1 = orc_tidal(per_d, m1, m2, ecc, incl, argp, nu[k], r1, axis_rs, mu1, tau1);
        double x1 = orc_irradiation(per_d, m1, m2, ecc, incl, argp, nu[k], r2, ref1);
        double f1 = w1 * (1 + b1 + e1 + x1);

        double b2 = orc_doppler(per_d, m2, m1, ecc, incl, (argp + K_PI), nu[k], ab2);
        double e2 = orc_tidal(per_d, m2, m1, ecc, incl, (argp + K_PI), nu[k], r2, axis_rs, mu2, tau2);
        double x2 = orc_irradiation(per_d, m2, m1, ecc, incl, (argp + K_PI), nu[k], r1, ref2);
        double f2 = w2 * (1 + b2 + e2 + x2);

        double ov = orc_overlap(r1, r2, sep[k]);
        if (z2[k] > z1[k]) f2 -= ov * w2 / (K_PI * (r2 * r2));
        else if (z2[k] < z1[k]) f1 -= ov * w1 / (K_PI * (r1 * r1));
        out[k] = (f1 + f2);
    }
    free(work);

    orc_median_shift(out, 0, n);
    for (int k = 0; k < n; ++k) {
        out[k] += 1;
        out[k] = (1 * blend + out[k] * (1 - blend)) * tune;
    }
}

/* ------------------------------------------------------------------ */
/* blackbody photometry (likelihood3.c:725-795)                         */
/* ------------------------------------------------------------------ */
void orc_photometry(const double *p, double dist, double *gmag, double *bmv,
                    double *vmg, double *gmt)
{
    double r1 = pow(10., orc_logrstar_table(p[0]) + p[7] * orc_radius_spread(p[0]));
    double r2 = pow(10., orc_logrstar_table(p[1]) + p[8] * orc_radius_spread(p[1]));
    double t1 = pow(10., orc_logteff_table(p[0]) + p[17] * orc_teff_spread(p[0]));
    double t2 = pow(10., orc_logteff_table(p[1]) + p[18] * orc_teff_spread(p[1]));
    r1 *= K_RSUN;
    r2 *= K_RSUN;

    static const double lam[4] = {442, 540, 673, 750};
    const double hp = 6.626e-27, kb = 1.38e-16, pc = 3.086e18;
    double blend = p[19];
    double fl[4];
    for (int k = 0; k < 4; ++k) {
        double fr = K_CLIGHT / (lam[k] * 1e-7);
        double pre = 2. * hp * ((fr * fr) * fr) / (K_CLIGHT * K_CLIGHT);
        fl[k] = K_PI * (r1 * r1 * (pre / (exp(hp * fr / (kb * t1)) - 1.))
                        + r2 * r2 * (pre / (exp(hp * fr / (kb * t2)) - 1.)))
                / ((dist * dist) * (pc * pc));
        fl[k] = fl[k] / (1 - blend);
    }
    double mb = -2.5 * log10(fl[0]) - 48.6;
    double mv = -2.5 * log10(fl[1]) - 48.6;
    double mg = -2.5 * log10(fl[2]) - 48.6;
    double mt = -2.5 * log10(fl[3]) - 48.6;
    *gmag = mg;
    *bmv = mb - mv;
    *vmg = mv - mg;
    *gmt = mg - mt;
}

/* ------------------------------------------------------------------ */
/* Roche-lobe overflow, Eggleton 1983 (likelihood3.c:945-974)            */
/* ------------------------------------------------------------------ */
double orc_lobe_fraction(double q)
{
    return 0.49 * pow(q, 2. / 3) / (0.6 * pow(q, 2. / 3) + log(1 + pow(q, 1. / 3)));
}

int orc_roche_flag(const double *p)
{
    double ma = pow(10., p[0]) * K_MSUN;
    double mb = pow(10., p[1]) * K_MSUN;
    double q = ma / mb;
    double per = pow(10., p[2]) * K_DAY;
    double ecc = p[3];
    double ra = pow(10., orc_logrstar_table(p[0]) + p[7] * orc_radius_spread(p[0])) * K_RSUN;
    double rb = pow(10., orc_logrstar_table(p[1]) + p[8] * orc_radius_spread(p[1])) * K_RSUN;
    double sep = pow(K_GRAV * (ma + mb) * (per * per) / (4.0 * K_PI * K_PI), 1. / 3.);
    double la = orc_lobe_fraction(q);
    double lb = orc_lobe_fraction(1 / q);
    double fa = ra / (sep * (1 - ecc));
    double fb = rb / (sep * (1 - ecc));
    return ((la < fa) || (lb < fb)) ? 1 : 0;
}

/* ------------------------------------------------------------------ */
/* log-likelihood (likelihood3.c:809-873).  Mutates sig[] exactly like    */
/* the reference: sigma < 1e-5 is clamped to 1e-5 in the caller's array.  */
/* ------------------------------------------------------------------ */
double orc_loglike(const double *tt, const double *flux, double *sig, long n,
                   const double *p, const double *mag, const double *magerr)
{
    double *model = (double *)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    orc_light_curve(tt, n, p, model);
    double chi2 = 0.;
    for (long k = 0; k < n; ++k) {
        if (sig[k] < 1.e-5) sig[k] = 1.e-5;
        double res = (model[k] - flux[k]) / sig[k];
        chi2 += res * res;
    }
    free(model);

    double g, c1, c2, c3;
    orc_photometry(p, mag[0], &g, &c1, &c2, &c3);
    double res = (g - mag[1]) / magerr[0];
    chi2 += res * res;

    if (orc_roche_flag(p)) chi2 = K_HUGE;
    return (-chi2 / 2.0);
}

/* Batched CPU baseline: W walkers (row-major W x 21) over one light curve.
 * sigma is clamped once up front (same values every call sees; removes the
 * reference's benign write race).  OpenMP over walkers, like
 * mcmc_wrapper2.c:383.  nthreads <= 0 keeps the OpenMP default. */
#ifdef _OPENMP
#include <omp.h>
#endif
void orc_loglike_batch(const double *tt, const double *flux, double *sig, long n,
                       const double *pw, long w, const double *mag, const double *magerr,
                       double *out, int nthreads)
{
    for (long k = 0; k < n; ++k)
        if (sig[k] < 1.e-5) sig[k] = 1.e-5;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (long j = 0; j < w; ++j) out[j] = orc_loglike(tt, flux, sig, n, pw + 21 * j, mag, magerr);
}

/* batched light curves, row-major W x N output */
void orc_light_curve_batch(const double *tt, long n, const double *pw, long w, double *out,
                           int nthreads)
{
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (long j = 0; j < w; ++j) orc_light_curve(tt, n, pw + 21 * j, out + n * j);
}

/* ------------------------------------------------------------------ */
/* model light curve over 30 d + one period, to a text file             */
/* (likelihood3.c:880-941, SAVECOMP = 0 as configured in likelihood3.h:30)*/
/* ------------------------------------------------------------------ */
void orc_write_lc_file(const double *p, const char *path)
{
    enum { NT = 10000 };
    double span = 30. + pow(10., p[2]);
    double step = span / (double)NT;
    double *tt = (double *)malloc(2 * NT * sizeof(double));
    double *lc = tt + NT;
    tt[0] = 0.;
    for (int i = 1; i < NT; ++i) tt[i] = tt[i - 1] + step; /* running sum, as written */
    orc_light_curve(tt, NT, p, lc);
    FILE *fp = fopen(path, "w");
    if (fp) {
        for (int i = 0; i < NT; ++i) fprintf(fp, "%12.5e\t%12.5e\n", tt[i], lc[i]);
        fclose(fp);
    }
    free(tt);
}
