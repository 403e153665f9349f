"""GPU parity: libhbmi.so (HIP, gfx950) against the reference's golden vectors
and the oracle, through the C-ABI.

Tolerances (fp64; the model is re-associated on the GPU):
  * logL: |gpu - ref| <= LOGL_RTOL * max(1, |ref|)  with LOGL_RTOL = 1e-10
    (BASELINE.json north_star); the Roche sentinel -5e14 must match exactly
    and NaN must map to NaN.
  * model light curves: |gpu - ref| <= max(1e-12 * max(1, (0.2/(1-e))^3),
    1e-11 * |ref|): absolute for values ~1; relative for large templates,
    which occur only at e > 0.85 near periastron (flux ~1e3 at e = 0.97),
    where the reference's own five Newton steps have not converged and its
    template is that unconverged iterate.  The factor is the model's own conditioning near periastron
    (beta <= 1/(1-e) enters up to beta^5 and dE/dM = 1/(1-e cos E)): for
    e <= 0.8 it is 1e-12; at e = 0.93 an ulp of the mean anomaly already moves
    the reference's own template by ~1e-11.
  * scalar entry points: relative 1e-12 (absolute 1e-15 near zero).
  * integer/index work (median rank, sort order, partition, Roche flag): exact.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

LOGL_RTOL = 1e-10
LC_ATOL = 1e-12
LC_RTOL_BIG = 1e-11
SC_RTOL = 1e-12
PD = C.POINTER(C.c_double)


def p(a):
    return a.ctypes.data_as(PD)


def close_logl(gpu, ref):
    gpu, ref = np.asarray(gpu), np.asarray(ref)
    assert gpu.shape == ref.shape
    nan_r, nan_g = np.isnan(ref), np.isnan(gpu)
    assert np.array_equal(nan_r, nan_g), "NaN pattern differs"
    sent = ref == -5e14
    assert np.array_equal(gpu[sent], ref[sent]), "Roche sentinel must be exact"
    ok = ~nan_r
    err = np.abs(gpu[ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
    assert err.max(initial=0.0) <= LOGL_RTOL, f"max rel err {err.max():.3e}"
    return err.max(initial=0.0)


def lc_tol(ecc, ref=None):
    ecc = np.clip(np.asarray(ecc, dtype=float), 0.0, 0.999)
    tol = LC_ATOL * np.maximum(1.0, (0.2 / (1.0 - ecc)) ** 3)
    if ref is None:
        return tol
    return np.maximum(tol[:, None], LC_RTOL_BIG * np.abs(ref))


def close_rel(gpu, ref, rtol=SC_RTOL, atol=1e-15):
    gpu, ref = np.asarray(gpu, dtype=float), np.asarray(ref, dtype=float)
    assert np.array_equal(np.isnan(gpu), np.isnan(ref))
    ok = ~np.isnan(ref)
    err = np.abs(gpu[ok] - ref[ok])
    lim = np.maximum(rtol * np.abs(ref[ok]), atol)
    assert (err <= lim).all(), f"worst {np.max(err / np.maximum(np.abs(ref[ok]), 1e-300)):.3e}"


# ---------------------------------------------------------------- scalars
def test_scalar_entry_points(hbmi):
    g = golden("scalars.npz")
    close_rel([hbmi.get_alpha_beam(x) for x in g["ab_in"]], g["ab_out"])
    close_rel([hbmi._getT(x) for x in g["lm_in"]], g["getT_out"])
    close_rel([hbmi._getR(x) for x in g["lm_in"]], g["getR_out"])
    close_rel([hbmi.envelope_Temp(x) for x in g["lm_in"]], g["envT_out"])
    close_rel([hbmi.envelope_Radius(x) for x in g["lm_in"]], g["envR_out"])
    close_rel([hbmi.Eggleton_RL(x) for x in g["egg_in"]], g["egg_out"])
    close_rel([hbmi.beaming(*r) for r in g["beam_in"]], g["beam_out"], rtol=1e-11, atol=1e-18)
    close_rel([hbmi.ellipsoidal(*r) for r in g["ell_in"]], g["ell_out"], rtol=1e-11, atol=1e-18)
    close_rel([hbmi.reflection(*r) for r in g["refl_in"]], g["refl_out"], rtol=1e-11, atol=1e-18)
    close_rel([hbmi.eclipse_area(*r) for r in g["ecl_in"]], g["ecl_out"], rtol=1e-10, atol=1e-12)


def test_stellar_mags_roche(hbmi):
    g = golden("scalars.npz")
    radii, mags, roche = [], [], []
    for pv, d in zip(g["pv"], g["dist"]):
        pv = np.ascontiguousarray(pv)
        o = [C.c_double() for _ in range(4)]
        hbmi.calc_radii_and_Teffs(p(pv), *[C.byref(x) for x in o])
        radii.append([x.value for x in o])
        hbmi.calc_mags(p(pv), float(d), *[C.byref(x) for x in o])
        mags.append([x.value for x in o])
        roche.append(hbmi.RocheOverflow(p(pv)))
    close_rel(radii, g["radii_out"])
    close_rel(mags, g["mags_out"], rtol=1e-12, atol=1e-12)
    assert np.array_equal(roche, g["roche_out"])


def test_traj(hbmi):
    g = golden("traj.npz")

    def run(times, tp):
        times = np.ascontiguousarray(times)
        tp = np.ascontiguousarray(tp)
        outs = [np.empty(len(times)) for _ in range(5)]
        hbmi.traj(p(times), p(tp), *[p(o) for o in outs], len(times))
        return outs

    def check(outs, ref):
        d, z1, z2, rr, ff = outs
        scale = np.abs(ref[3]).max()
        for got, want in ((d, ref[0]), (z1, ref[1]), (z2, ref[2]), (rr, ref[3])):
            assert np.abs(got - want).max() <= 1e-12 * scale
        dphi = np.angle(np.exp(1j * (ff - ref[4])))
        assert np.abs(dphi).max() <= 1e-11

    check(run(g["times"], g["tp"]), [g["d"], g["z1"], g["z2"], g["rr"], g["ff"]])
    for tp, ex in zip(g["ex_tp"], g["ex_out"]):
        check(run(g["ex_times"], tp), ex)


def test_median_sort_partition_exact(hbmi):
    g = golden("median.npz")
    for i in range(int(g["ncases"][0])):
        a = g[f"in{i}"].copy()
        hbmi.remove_median(p(a), 0, len(a))
        assert np.array_equal(a, g[f"rm{i}"]), i
        b = g[f"in{i}"].copy()
        hbmi.quickSort(p(b), 0, len(b) - 1)
        assert np.array_equal(b, g[f"qs{i}"]), i  # -0.0 == 0.0 compares equal
        c = g[f"in{i}"].copy()
        k = hbmi.partition(p(c), 0, len(c) - 1)
        assert int(k) == int(g[f"pk{i}"][0]) and np.array_equal(c, g[f"pa{i}"]), i


# ------------------------------------------------------ light curve / logL
LC_FIXTURES = ["lc_synth1024.npz", "lc_synth7.npz", "lc_real231937440.npz"]


@pytest.mark.parametrize("latency", [True, False], ids=["small-batch-plan", "one-wave-plan"])
@pytest.mark.parametrize("name", LC_FIXTURES)
def test_batched_templates_and_logl(hbmi, name, latency):
    """Small batches take the multi-wave latency plan by default; the one-wave
    kernel (every batch of 512+ walkers) is checked on the same goldens."""
    from hb_mcmc_amd.likelihood import HBLikelihood

    g = golden(name)
    with HBLikelihood(g["t"], g["f"], g["s"], g["mag"], g["magerr"], latency_plan=latency) as L:
        tm = L.light_curve(g["params"])
        ll = L.loglike(g["params"])
    ref_t = g["templates"]
    bad = np.isnan(ref_t).any(1)
    assert np.array_equal(np.isnan(tm).any(1), bad)
    dev = np.abs(tm - ref_t).max(1)
    tol = lc_tol(g["params"][:, 3])
    worst = int(np.nanargmax(np.where(bad, -1, dev / tol)))
    assert (dev[~bad] <= tol[~bad]).all(), (f"walker {worst}: max |dt| {dev[worst]:.3e} > {tol[worst]:.1e}, "
                                            f"e={g['params'][worst, 3]:.4f}")
    close_logl(ll, g["logl"])


def test_n20000_lds_tiled_path(hbmi):
    from hb_mcmc_amd.likelihood import HBLikelihood

    g = golden("lc_synth20000.npz")
    with HBLikelihood(g["t"], g["f"], g["s"], g["mag"], g["magerr"]) as L:
        assert L.waves_per_walker == 16 and L.template_in_lds
        assert L.eval_kernel == "hb_eval_block_kernel"
        ll = L.loglike(g["params"])
        tm = L.light_curve(g["params"])
    close_logl(ll, g["logl"])
    tol = lc_tol(g["params"][:, 3])[:, None]
    assert (np.abs(tm[:, :16] - g["thead"]) <= tol).all()
    assert (np.abs(tm[:, -16:] - g["ttail"]) <= tol).all()
    assert (np.abs(tm.sum(1) - g["tsum"]) <= 20000 * tol[:, 0]).all()


def mean_anomaly_cond(oracle, t, P):
    """Per cadence, what one ulp of the mean anomaly moves the reference's own
    template by: |d template / dM| * 2^-52 * max(1, |M|), M = 2 pi (t - T0) / P
    (the reference rounds 2 pi (t DAY - T0 DAY) / (P DAY), likelihood3.c:147-150,
    before its Newton steps).  d/dM from a central difference of the oracle's
    light curve.  Near periastron at high e this is the model's conditioning:
    beta = 1/(1 - e cos E) enters up to beta^5 and dE/dM = beta."""
    Pd = 10.0 ** P[:, 2]
    out = np.empty((len(P), len(t)))
    for w in range(len(P)):
        h = 1e-6 * Pd[w]
        d = (oracle.light_curve(t + h, P[w]) - oracle.light_curve(t - h, P[w])) / (2.0 * h)
        M = 2.0 * np.pi * (t - P[w, 6]) / Pd[w]
        out[w] = np.abs(d) * Pd[w] / (2.0 * np.pi) * 2.0 ** -52 * np.maximum(1.0, np.abs(M))
    return out


def ulp_sensitivity(oracle, t, P, ref):
    """Per cadence, how far the reference's own template moves when the
    cadence's mean anomaly moves by one ulp (up or down): its discrete
    ill-conditioning, which the derivative above misses -- e.g. an eclipse
    near the regime boundary of eclipse_area (likelihood3.c:353-389), where
    asin is evaluated next to 1 (at N = 4096, e = 0.85 the reference's values
    at two cadences of the same phase, one period apart, differ by 3.2e-12).
    The shift is dt = max(ulp(t), ulp(M) P / 2 pi): one ulp of the time, or
    of M where that is coarser (early cadences, |t| << |M| P / 2 pi: at N =
    6001, t = 0.068 d, M = -4.4, one ulp of M moves the reference's template
    by 6.3e-12 and one ulp of t by 2.2e-16) -- any solver's E carries M's
    rounding, whatever its Newton path."""
    Pd = 10.0 ** P[:, 2]
    M = 2.0 * np.pi * (t[None, :] - P[:, 6:7]) / Pd[:, None]
    dt = np.maximum(np.spacing(np.abs(t))[None, :], np.spacing(np.abs(M)) * Pd[:, None] / (2.0 * np.pi))
    out = np.empty_like(ref)
    for w in range(len(P)):
        up = oracle.light_curve(t + dt[w], P[w])
        dn = oracle.light_curve(t - dt[w], P[w])
        out[w] = np.maximum(np.abs(up - ref[w]), np.abs(dn - ref[w]))
    return out


# The cold Kepler path at e >= 0.85 (scripts/cold_err_probe.py, GPU, N = 2048
# .. 4096, sorted and shuffled cadences, one-wave / pair / rows plans,
# profiles/r04/r04a_cold_err_probe*.log): the template error is at most 1.4 x
# mean_anomaly_cond, except at one cadence pair (N = 4096, e = 0.85: 4.35e-12,
# the same on the rows and the block kernel, profiles/r04/r04c_cold_err_where_*),
# where it is 2.7 x ulp_sensitivity.  Bounds: 4 x mean_anomaly_cond, and
# K_ULP x ulp_sensitivity per plan from what each needs (check_cold's record,
# profiles/r06/r06d_kulp.jsonl, round 6): the pair, rows and one-wave plans
# none (every cadence inside the other two terms), the block kernel 1.71 (N =
# 6001) and 1.41 (N = 20 000) -- so 2 and 4 (round 5: 8 everywhere).
K_COND = 4.0
K_ULP = 4.0          # block kernel (and tests that mix it in)
K_ULP_WAVES = 2.0    # one-wave, pair and rows plans


def check_cold(oracle, t, P, ref, tm, label, k_ulp=K_ULP):
    """Templates under the conditioning bound; with HB_TEST_KULP_LOG set, also record the
    smallest K_ULP this case needs (0: the eccentricity-scaled bound and the
    conditioning term cover every cadence), so the factor's margin on each
    plan is on file (profiles/r06/r06*_kulp.jsonl)."""
    ok = ~np.isnan(ref).any(1)
    base = np.maximum(lc_tol(P[:, 3], ref), K_COND * mean_anomaly_cond(oracle, t, P))
    ulp = ulp_sensitivity(oracle, t, P, ref)
    tol = np.maximum(base, k_ulp * ulp)
    err = np.abs(tm - ref)
    worst = np.nanmax(np.where(ok[:, None], err / tol, 0.0))
    log = os.environ.get("HB_TEST_KULP_LOG")
    if log:
        over = ok[:, None] & (err > base)
        need = float(np.max(np.where(over, err / np.maximum(ulp, 1e-300), 0.0))) if over.any() else 0.0
        with open(log, "a") as fp:
            fp.write(json.dumps({"case": label, "k_ulp_needed": need, "cadences_over_base": int(over.sum()),
                                 "worst_over_bound": float(worst)}) + "\n")
    assert worst <= 1.0, f"template error {worst:.2f} x the bound"


@pytest.mark.parametrize("n", [2049, 3000, 4001, 4096, 4097, 6001, 8192, 12000])
def test_block_kernel_sizes(hbmi, oracle, n):
    """N = 2049..4096: the rows kernel (4 waves of lane rows per walker);
    above, the register-key block kernel across its (waves, keys-per-thread)
    classes.  Odd and even N (median rank likelihood3.c:97-101), templates
    and logL; each walker bit-identical when the batch is reversed."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.walkers(8, seed=n)
    with HBLikelihood(t, f, s) as L:
        assert L.eval_kernel == ("hb_eval_wave_kernel" if n <= 4096 else "hb_eval_block_kernel")
        ll = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P)
    assert np.array_equal(ll, rev, equal_nan=True)
    close_logl(ll, oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))
    ref = oracle.light_curve_batch(t, P, 8)
    tol = lc_tol(P[:, 3])[:, None]
    assert (np.abs(tm - ref) <= tol).all()


@pytest.mark.parametrize("n", [1280, 1281, 1500, 2047, 2048])
def test_pair_plan_sizes(hbmi, oracle, n):
    """N = 1281..2048 runs a pair of waves per walker (1280 is
    the last one-wave size): templates and logL against the oracle, with
    walkers on the cold Kepler path (e = 0.85 and 0.9: the pair's cold pass
    writes cadences of either wave's rows) and Roche walkers; and every walker's logL
    bit-identical when the batch is evaluated again in reversed order (the
    pair's LDS hand-overs are race-free)."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.walkers(64, seed=n)
    P[::4, 3] = 0.9  # cold path (e > 0.8)
    P[2::8, 3] = 0.85
    with HBLikelihood(t, f, s) as L:
        assert L.eval_kernel == "hb_eval_wave_kernel"
        ll = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P)
    assert np.array_equal(ll, rev, equal_nan=True)
    close_logl(ll, oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))
    ref = oracle.light_curve_batch(t, P, 8)
    # the eccentricity-scaled bound, or at high e the model's own conditioning
    # (check_cold: derived from the measured errors, not a blanket bound)
    check_cold(oracle, t, P, ref, tm, f"pair-{n}", K_ULP_WAVES)


@pytest.mark.parametrize("order", ["sorted", "shuffled"])
@pytest.mark.parametrize("n", [2049, 3000, 4096])
def test_rows_plan_cold_roche_shuffled(hbmi, oracle, n, order):
    """N = 2049..4096 runs four waves of lane rows per walker (the rows kernel).
    64 walkers with Roche walkers (logL sentinel, no model pass), cold walkers
    at e = 0.85 and 0.9 (model_pass_cold: each wave writes cadences of the other
    waves' rows, and their eclipse terms land there too), and a shuffled cadence
    order (the warm-chain gate then sends every walker to the cold pass):
    templates and logL against the oracle, and every walker's logL bit-identical
    when the batch is evaluated again in reversed order."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    if order == "shuffled":
        p = np.random.default_rng(n).permutation(n)
        t, f, s = t[p], f[p], s[p]
    P = synth.walkers(64, seed=n, roche_frac=0.1)
    P[0::8, 3] = 0.85
    P[4::8, 3] = 0.9
    with HBLikelihood(t, f, s) as L:
        assert L.eval_kernel == "hb_eval_wave_kernel" and L.waves_per_walker == 4
        ll = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P)
    assert np.array_equal(ll, rev, equal_nan=True)
    ref_ll = oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    close_logl(ll, ref_ll)
    assert (ref_ll == -5e14).sum() >= 3  # Roche walkers present (sentinel exact in close_logl)
    ref = oracle.light_curve_batch(t, P, 8)
    check_cold(oracle, t, P, ref, tm, f"rows-{n}-{order}", K_ULP_WAVES)


@pytest.mark.parametrize("order", ["sorted", "shuffled"])
@pytest.mark.parametrize("n", [4097, 6001, 12000, 20000])
def test_block_kernel_cold_roche_shuffled(hbmi, oracle, n, order):
    """N > 4096 runs the block kernel (every (waves, keys-per-thread) class it
    takes up to C3's N = 20 000): 64 walkers with Roche walkers, e = 0.85 /
    0.9 walkers beside the usual ones, sorted and shuffled cadence orders;
    templates and logL against the oracle under the conditioning bound, and
    every walker's logL bit-identical when the batch is evaluated in
    reverse."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    if order == "shuffled":
        p = np.random.default_rng(n).permutation(n)
        t, f, s = t[p], f[p], s[p]
    P = synth.walkers(64, seed=n + 1, roche_frac=0.1)
    P[0::8, 3] = 0.85
    P[4::8, 3] = 0.9
    with HBLikelihood(t, f, s) as L:
        assert L.eval_kernel == "hb_eval_block_kernel"
        ll = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P)
    assert np.array_equal(ll, rev, equal_nan=True)
    ref_ll = oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    close_logl(ll, ref_ll)
    assert (ref_ll == -5e14).sum() >= 3  # Roche walkers present
    ref = oracle.light_curve_batch(t, P, 8)
    check_cold(oracle, t, P, ref, tm, f"block-{n}-{order}")


@pytest.mark.parametrize("n,order", [(6001, "sorted"), (1024, "shuffled"), (200, "sorted"), (1024, "sorted"),
                                     (1500, "sorted"), (3000, "sorted")],
                         ids=["block-kernel", "one-wave-cold", "one-wave-vpt4", "one-wave-warm", "pair", "rows"])
def test_series_kepler_start_boundary(hbmi, oracle, n, order):
    """The cold path's series Kepler start (hb_device.hpp cold_start_k, |e| <=
    kSeriesEmax = 0.25 on the phase table) and the reference's start on either
    side of its bound, e = 0 and negative e included: the block kernel (N =
    6001), the one-wave cold pass (shuffled cadences leave the warm-chain gate)
    and a 4-cadence-per-lane light curve, and the warm chains (sorted N =
    1024); templates under the conditioning bound and logL against the
    oracle, batch reversal bit-identical.  Negative e is Kepler's equation at
    M + pi: the Newton stopping rule and the warm-chain gate take |e| (with e
    itself the rule stopped after one step for every e < 0: logL off by up to
    3e-3 before round 5's fix)."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    if order == "shuffled":
        p = np.random.default_rng(n + 7).permutation(n)
        t, f, s = t[p], f[p], s[p]
    es = [0.0, 1e-9, 0.05, 0.1, 0.226, 0.24, 0.2499, 0.25, np.nextafter(0.25, 1.0), 0.2501, 0.3, 0.6,
          -0.1, -0.25, -0.2501, 0.85]
    P = synth.walkers(len(es), seed=n + 5, roche_frac=0.0)
    P[:, 3] = es
    with HBLikelihood(t, f, s) as L:
        ll = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P)
    assert np.array_equal(ll, rev, equal_nan=True)
    close_logl(ll, oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))
    ref = oracle.light_curve_batch(t, P, 8)
    ok = ~np.isnan(ref).any(1)
    assert ok.sum() >= len(es) - 2
    check_cold(oracle, t, P, ref, tm, f"series-boundary-{n}-{order}")


KEPLER_ES = [0.0, 1e-9, 0.01, 0.05, 0.1, 0.15, 0.2, 0.226, 0.24, 0.2499, 0.25, -0.05, -0.1, -0.226, -0.25]


@pytest.mark.parametrize("tab", [1, 0], ids=["table-series-start", "direct-reference-start"])
def test_kepler_cold_start_against_reference_root(hbmi, oracle, tab):
    """The series Kepler start pinned at the solver, not only through the
    template envelope: the eval kernels' cold_start_k + newton_k (stopping
    rule included; hb_kepler_probe_kernel) on a dense grid of 2^20 mean
    anomalies over (-2 pi, 2 pi) plus the edges (+-pi, +-2pi, tiny |M|), for
    e in [-0.25, 0.25] and on both sides of the series gate (+-0.25 and the
    next doubles out), against the reference's five-step root
    (likelihood3.c:152-160, oracle.kepler).  tab=1: on the phase table (the
    series start for |e| <= 0.25, the reference's start by rotation outside);
    tab=0: the direct path (the reference's start).  Every lane converges and
    E agrees within 2 ulp of E on the series start (within 2^-57 absolute
    below |E| = 2^-6); the reference's start, outside the gate or off the
    table, within 12 ulp + 2^-54 absolute (its rotation-carried (sin, cos)
    hold a few 1e-16 absolute; measured <= 8.5 ulp).
    The stopping rule is a quarter ulp of E for the predicted next correction; rounds 1-5's absolute 2^-52 left up to
    3 ulp (e = 0.1, M = -0.41: 2.5 ulp from the true root where the
    reference's five steps are 0.46 ulp away)."""
    lib = hbmi
    two_pi = 2.0 * np.pi
    n = 1 << 20
    M = (np.arange(n) + 0.5) / n * (2.0 * two_pi) - two_pi  # symmetric, never 0
    edges = [np.pi, np.nextafter(np.pi, 0), np.nextafter(np.pi, 4), two_pi - 1e-12, np.nextafter(two_pi, 0),
             1e-300, 5e-324, 1e-8, 0.5 * np.pi, 1.5 * np.pi]
    M = np.concatenate([M, edges, [-x for x in edges]])
    es = KEPLER_ES + [np.nextafter(0.25, 1.0), -np.nextafter(0.25, 1.0), 0.2501, -0.2501]
    out = np.empty(4 * len(M))
    report = []
    for e in es:
        assert lib.hbx_kepler_probe(p(M), len(M), float(e), tab, p(out)) == 0
        got = out.reshape(-1, 4)
        assert (got[:, 1] == 1.0).all(), f"e={e}: {int((got[:, 1] != 1.0).sum())} lanes did not converge"
        ref = oracle.kepler(M, e)
        # the true root (x87 long double Newton from the reference's root):
        # both solvers' distance from it, for the record
        Ml, El, el = M.astype(np.longdouble), ref.astype(np.longdouble), np.longdouble(e)
        for _ in range(3):
            El = El - (El - el * np.sin(El) - Ml) / (1 - el * np.cos(El))
        sp = np.spacing(np.abs(ref))
        # the series start (on the table, |e| <= 0.25): 2 ulp of E, and 2^-57
        # absolute below |E| = 2^-6.  The reference's start (outside the gate,
        # or off the table) is 0.85 e from the root and reaches it through
        # three or four steps of wide rotations / sincos_fast, whose (sin,
        # cos) carry a few 1e-16 absolute: measured up to 8.5 ulp of E from
        # the true root (6.9e-16 absolute), against the reference's 1.2 --
        # bound 12 ulp + 2^-54 (template effect < 1e-15, the budget is 1e-12)
        big = np.abs(ref) >= 2.0 ** -6
        series = tab == 1 and abs(e) <= 0.25
        tol = np.where(big, 2.0 * sp, 2.0 * sp + 2.0 ** -57) if series else 12.0 * sp + 2.0 ** -54
        dev = np.abs(got[:, 0] - ref)
        i = int(np.argmax(dev / tol))
        vs_root = np.abs((got[:, 0] - El).astype(np.float64))
        report.append({"e": e, "max_ulp_vs_reference": float(np.max(dev[big] / sp[big])),
                       "max_ulp_vs_root": float(np.max(vs_root[big] / sp[big])),
                       "reference_max_ulp_vs_root": float(np.max(np.abs((ref - El).astype(np.float64))[big] / sp[big])),
                       "max_abs_vs_reference_small_E": float(np.max(dev[~big]))})
        log = os.environ.get("HB_TEST_KULP_LOG")
        if log:
            with open(log, "a") as fp:
                fp.write(json.dumps({"case": f"kepler-probe-tab{tab}", **report[-1]}) + "\n")
        assert dev[i] <= tol[i], (f"e={e}: E off by {dev[i] / sp[i]:.1f} ulp at M={M[i]!r} "
                                  f"({got[i, 0]!r} vs {ref[i]!r})")
        # (sin, cos)(E) carried by the rotations: within a few ulp of libm's
        assert np.abs(got[:, 2] - np.sin(got[:, 0])).max() <= 4e-15
        assert np.abs(got[:, 3] - np.cos(got[:, 0])).max() <= 4e-15


@pytest.mark.parametrize("latency", [True, False], ids=["small-batch-plan", "one-wave-plan"])
@pytest.mark.parametrize("n", [1024, 6001])
def test_phase_table_and_direct_paths(hbmi, oracle, n, latency):
    """Walkers on the batch's table period (walker 0's P) take the phase-table
    Kepler start, the others the direct sincos; both against the oracle, and a
    walker's logL agrees whichever path it takes.  T0 = 0 and T0 = t_k put
    cadences exactly on x = 0 (the exact-fmod branch)."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.walkers(48, seed=11, roche_frac=0.0)
    P[1::3, 2] += 1e-3 * np.random.default_rng(4).standard_normal(len(P[1::3]))  # off the table period
    P[3, 6] = 0.0
    P[6, 6] = t[5]
    P[9, 3] = 0.6  # larger steps: direct sincos inside the Newton loop
    Q = P.copy()
    Q[0, 2] += 2e-3  # walker 0 moves: now every other walker is off the table period
    with HBLikelihood(t, f, s, latency_plan=latency) as L:
        a = L.loglike(P)
        b = L.loglike(Q)
        tm = L.light_curve(P)
    ref = oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    close_logl(a, ref)
    close_logl(b[1:], ref[1:])
    tol = lc_tol(P[:, 3])[:, None]
    assert (np.abs(tm - oracle.light_curve_batch(t, P, 8)) <= tol).all()


@pytest.mark.parametrize("latency", [True, False], ids=["small-batch-plan", "one-wave-plan"])
def test_real_1861_cadences(hbmi, latency):
    from hb_mcmc_amd.likelihood import HBLikelihood

    g = golden("lc_real237957506.npz")
    with HBLikelihood(g["t"], g["f"], g["s"], g["mag"], g["magerr"], latency_plan=latency) as L:
        close_logl(L.loglike(g["params"]), g["logl"])


def test_hbm_scratch_path(hbmi, oracle):
    """N beyond the LDS budget: template slab in HBM."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    n = 24000
    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.walkers(6, seed=5)
    with HBLikelihood(t, f, s) as L:
        assert not L.template_in_lds
        close_logl(L.loglike(P), oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))


def test_dropin_loglikelihood_mutates_noise(hbmi):
    g = golden("lc_synth1024.npz")
    t, f = g["t"].copy(), g["f"].copy()
    s = g["s"].copy()
    mag, err = g["mag"].copy(), g["magerr"].copy()
    got = []
    for pv in g["params"][:6]:
        pv = pv.copy()
        got.append(hbmi.loglikelihood(p(t), p(f), p(s), len(t), p(pv), p(mag), p(err)))
    assert np.array_equal(s, np.maximum(g["s"], 1e-5))  # likelihood3.c:824-827 side effect
    close_logl(got, g["logl"][:6])
    out = np.empty(len(t))
    pv = g["params"][0].copy()
    hbmi.calc_light_curve(p(t), len(t), p(pv), p(out))
    assert np.abs(out - g["templates"][0]).max() <= lc_tol(pv[3])


def test_dropin_concurrent_calls_are_combined_exactly(hbmi):
    """The drop-in combines concurrent loglikelihood() calls on one light curve
    into batched launches (hb_capi.hip dropin_loglik): 16 threads x 24 calls
    (ctypes releases the GIL) give each caller exactly the value a lone call
    gives, and two light curves in flight at once keep their own contexts."""
    import threading

    g = golden("lc_synth1024.npz")
    t, f, s = g["t"].copy(), g["f"].copy(), g["s"].copy()
    t2 = t[:883].copy()
    f2, s2 = f[:883].copy(), s[:883].copy()
    mag, err = g["mag"].copy(), g["magerr"].copy()
    P = np.ascontiguousarray(g["params"][:24])
    solo = [hbmi.loglikelihood(p(t), p(f), p(s), len(t), p(P[i].copy()), p(mag), p(err)) for i in range(24)]
    solo2 = [hbmi.loglikelihood(p(t2), p(f2), p(s2), len(t2), p(P[i].copy()), p(mag), p(err)) for i in range(24)]
    res, res2, errs = {}, {}, []
    # with the logL memo on, every threaded call below would be answered from
    # the table; off, they are combined into launches
    hbmi.hbx_dropin_set_memo(0)

    def worker(k):
        try:
            for r in range(24):
                i = (k * 7 + r) % 24
                pv = P[i].copy()
                if (k + r) % 3 == 0:
                    res2[(k, r)] = (i, hbmi.loglikelihood(p(t2), p(f2), p(s2), len(t2), p(pv), p(mag), p(err)))
                else:
                    res[(k, r)] = (i, hbmi.loglikelihood(p(t), p(f), p(s), len(t), p(pv), p(mag), p(err)))
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(16)]
    try:
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        hbmi.hbx_dropin_set_memo(1)
    assert not errs
    assert len(res) + len(res2) == 16 * 24
    for i, v in res.values():
        assert v == solo[i] or (np.isnan(v) and np.isnan(solo[i]))
    for i, v in res2.values():
        assert v == solo2[i] or (np.isnan(v) and np.isnan(solo2[i]))
    close_logl(solo, g["logl"][:24])


def _dropin_stats(hbmi):
    out = np.zeros(11)
    assert hbmi.hbx_dropin_stats(p(out), 11) == 11
    return dict(zip(("calls", "memo_hits", "batches", "walkers", "max_batch", "created"), out[:6]))


def test_dropin_memo_hit_and_bit_flip(hbmi):
    """mcmc_wrapper2.c:488 re-asks for logL of x[chain_id], a state the library
    has evaluated already: the drop-in answers it from the context's memo
    (exact parameter bytes) without a launch.  One flipped mantissa bit is a
    fresh evaluation, and every value equals the batched API's for the same
    vector bit for bit.  A second light curve one ulp away gets its own
    context and memo."""
    from hb_mcmc_amd.likelihood import HBLikelihood

    g = golden("lc_synth1024.npz")
    t, s = g["t"].copy(), g["s"].copy()
    f = g["f"].copy()
    f[5] = np.nextafter(f[5], 2.0)  # a light curve no earlier test used: a fresh context
    mag, err = g["mag"].copy(), g["magerr"].copy()
    P = np.ascontiguousarray(g["params"][:3]).copy()
    q = P[1].copy()
    q.view(np.uint64)[4] ^= np.uint64(1)  # lowest mantissa bit of the inclination
    with HBLikelihood(t, f, np.maximum(s, 1e-5), g["mag"], g["magerr"]) as L:
        want = L.loglike(np.vstack([P, q[None, :]]))
    s0 = _dropin_stats(hbmi)
    v0 = hbmi.loglikelihood(p(t), p(f), p(s), len(t), p(P[1].copy()), p(mag), p(err))
    s1 = _dropin_stats(hbmi)
    assert s1["created"] == s0["created"] + 1 and s1["batches"] == s0["batches"] + 1
    v1 = hbmi.loglikelihood(p(t), p(f), p(s), len(t), p(P[1].copy()), p(mag), p(err))
    s2 = _dropin_stats(hbmi)
    assert s2["memo_hits"] == s1["memo_hits"] + 1 and s2["batches"] == s1["batches"]
    vq = hbmi.loglikelihood(p(t), p(f), p(s), len(t), p(q), p(mag), p(err))
    s3 = _dropin_stats(hbmi)
    assert s3["batches"] == s2["batches"] + 1 and s3["memo_hits"] == s2["memo_hits"]
    assert v0 == want[1] and v1 == want[1] and vq == want[3]
    # the other light curve (f one ulp apart at cadence 5) is its own context
    f0 = g["f"].copy()
    u = hbmi.loglikelihood(p(t), p(f0), p(s), len(t), p(P[1].copy()), p(mag), p(err))
    with HBLikelihood(t, f0, np.maximum(s, 1e-5), g["mag"], g["magerr"]) as L0:
        assert u == L0.loglike(P[1:2])[0]


def test_dropin_light_curves_on_one_hash_key_stay_apart(hbmi):
    """Every light curve forced onto one cache key (hbx_dropin_test_hash): two
    light curves that differ in one flux value still get two contexts, and
    each call evaluates its own arrays (the full compare behind a hash hit)."""
    from hb_mcmc_amd.likelihood import HBLikelihood

    g = golden("lc_synth1024.npz")
    t, s = g["t"].copy(), g["s"].copy()
    fa, fb = g["f"].copy(), g["f"].copy()
    fa[9] += 1e-3
    fb[9] -= 1e-3
    mag, err = g["mag"].copy(), g["magerr"].copy()
    pv = g["params"][2].copy()
    hbmi.hbx_dropin_test_hash(1)
    try:
        c0 = _dropin_stats(hbmi)["created"]
        va = hbmi.loglikelihood(p(t), p(fa), p(s), len(t), p(pv), p(mag), p(err))
        vb = hbmi.loglikelihood(p(t), p(fb), p(s), len(t), p(pv), p(mag), p(err))
        va2 = hbmi.loglikelihood(p(t), p(fa.copy()), p(s), len(t), p(pv), p(mag), p(err))
        assert _dropin_stats(hbmi)["created"] == c0 + 2
    finally:
        hbmi.hbx_dropin_test_hash(0)
    for fx, v in ((fa, va), (fb, vb), (fa, va2)):
        with HBLikelihood(t, fx, np.maximum(s, 1e-5), g["mag"], g["magerr"]) as L:
            assert v == L.loglike(pv[None, :])[0]
    assert va != vb


# ------------------------------------------------- fused launch
@pytest.mark.parametrize("n,w", [(1024, 4096), (1024, 2048), (1024, 1000), (1024, 5), (1024, 4097),
                                 (512, 4096), (100, 777), (7, 64)])
def test_fused_launch_equals_two_launches(hbmi, oracle, n, w):
    """hb_loglik_batch_dev makes ONE launch up to 16 walkers per CU (the
    records computed in the eval kernel's prologue, the phase table in LDS):
    bit-identical to the two-launch path (hb_prepare_dev + hb_evaluate_dev) on
    the same walkers, and it leaves the same records and global phase table
    behind (an hb_evaluate_dev right after it gives the same values again).
    Walkers off the table period, Roche walkers and cold (e = 0.85) walkers
    included; a sample against the oracle."""
    import torch

    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.walkers(w, seed=n + w)
    P[1::7, 2] += 1e-4  # off walker 0's period: direct sincos
    P[2::9, 3] = 0.85   # cold Kepler path
    dev = torch.device("cuda", 0)
    Pd = torch.from_numpy(P).to(dev)
    a, b, c = (torch.empty(w, dtype=torch.float64, device=dev) for _ in range(3))
    with HBLikelihood(t, f, s) as L:
        L.reserve(w)
        fw = L.fused_wpb(w)
        assert (fw > 0) == (n <= 1024 and w <= 4096), fw
        L.prepare_dev(Pd)
        L.evaluate_dev(w, a)
        L.loglike_dev(Pd, b)
        L.evaluate_dev(w, c)  # the records / table the fused launch left behind
        torch.cuda.synchronize()
    a, b, c = a.cpu().numpy(), b.cpu().numpy(), c.cpu().numpy()
    assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(b, c, equal_nan=True)
    idx = np.arange(0, w, max(1, w // 128))
    close_logl(b[idx], oracle.loglike_batch(t, f, s, P[idx], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))


@pytest.mark.parametrize("w", [4096, 333])
def test_fused_launch_phase_table_cache(hbmi, oracle, w):
    """A fused launch that follows a fused launch of the same table period
    loads the global phase table instead of computing it (fused_prologue,
    PreArgs::tab_prev).  A sequence on one context -- period A twice, a batch
    whose walker 0 has period B (the table is rebuilt), B again (cached), a
    two-launch prep with period A in between (the chain breaks), then A, A --
    gives every fused batch bit for bit the values of the two-launch path on
    a fresh context, and the table it leaves serves hb_evaluate_dev."""
    import torch

    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    n = 1024
    t, f, s = synth.dataset(n, oracle.light_curve)
    PA = synth.walkers(w, seed=71)
    PB = synth.walkers(w, seed=72)
    PB[:, 2] += 3e-4            # every walker on period B (the table period of its batch)
    PA[1::5, 2] += 1e-4         # a few off the table period: direct sincos
    dev = torch.device("cuda", 0)

    def two_launch(P):
        with HBLikelihood(t, f, s) as R:
            R.reserve(w)
            o = torch.empty(w, dtype=torch.float64, device=dev)
            R.prepare_dev(torch.from_numpy(P).to(dev))
            R.evaluate_dev(w, o)
            torch.cuda.synchronize()
            return o.cpu().numpy()

    want = {"A": two_launch(PA), "B": two_launch(PB)}
    seq = ["A", "A", "B", "B", "prepA", "A", "A", "B", "A"]
    with HBLikelihood(t, f, s) as L:
        L.reserve(w)
        assert L.fused_wpb(w) > 0
        for k, name in enumerate(seq):
            P = PA if name.endswith("A") else PB
            Pd = torch.from_numpy(P).to(dev)
            o = torch.empty(w, dtype=torch.float64, device=dev)
            if name.startswith("prep"):
                L.prepare_dev(Pd)
                L.evaluate_dev(w, o)
            else:
                L.loglike_dev(Pd, o)
            c = torch.empty(w, dtype=torch.float64, device=dev)
            L.evaluate_dev(w, c)  # the records and global table this launch left behind
            torch.cuda.synchronize()
            got, again = o.cpu().numpy(), c.cpu().numpy()
            ref = want[name[-1]]
            assert np.array_equal(got, ref, equal_nan=True), f"step {k} ({name})"
            assert np.array_equal(again, ref, equal_nan=True), f"step {k} ({name}): table left behind"


# ------------------------------------------------- full-size (config C2)
def test_full_size_c2_against_oracle_and_properties(hbmi, oracle):
    """W=4096, N=1024: oracle on a 256-walker sample; size-independent
    properties on all walkers (determinism, permutation equivariance, Roche)."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(1024, oracle.light_curve)
    P = synth.walkers(4096, seed=1)
    with HBLikelihood(t, f, s) as L:
        a = L.loglike(P)
        b = L.loglike(P)
        perm = np.random.default_rng(0).permutation(4096)
        c = L.loglike(P[perm])
    assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(a[perm], c, equal_nan=True)
    idx = np.arange(0, 4096, 16)
    ref = oracle.loglike_batch(t, f, s, P[idx], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    close_logl(a[idx], ref)
    roche = (a == -5e14)
    assert 0.02 < roche.mean() < 0.2
    assert np.isfinite(a[~roche]).all()


@pytest.mark.parametrize("seed", [11, 12])
def test_prior_spread_walkers_c2(hbmi, oracle, seed):
    """W = 4096, N = 1024 on walkers drawn from the set_limits box like the
    reference's random initial state (mcmc_wrapper2.c:236-252): e over
    [0, 1), masses over the whole prior range -- cold-path (e > 0.8) and
    Roche walkers, the spread the sampler's hot rungs feed the likelihood
    (the bench's c2_prior_spread key).  Every walker against the oracle (NaN
    pattern and Roche sentinel exact, 1e-10 relative otherwise), and each
    walker bit-identical when the batch is reversed."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(1024, oracle.light_curve)
    P = synth.prior_walkers(4096, seed=seed)
    with HBLikelihood(t, f, s) as L:
        a = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
    assert np.array_equal(a, rev, equal_nan=True)
    ref = oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    close_logl(a, ref)
    roche = ref == -5e14
    assert 0.3 < roche.mean() < 0.8
    assert ((P[:, 3] > 0.8) & ~roche).sum() >= 20  # cold-path walkers are exercised


@pytest.mark.parametrize("n", [1024, 1500, 3000, 20000])
def test_eccentricity_above_one_every_plan(hbmi, oracle, n):
    """Walkers with |e| > 1 (the sampler's hot rungs propose them: e has no
    upper wall, likelihood3.c:986-1121), and e = -1 exactly (1 - e^2 = 0), take
    logl_without_light_curve's NaN;
    e < -1 walkers in Roche overflow the sentinel.  One-wave, pair, rows and
    block plans against the oracle: NaN pattern and sentinel exact, the
    finite walkers beside them within 1e-10, and the batch reversed bit for
    bit."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.prior_walkers(48, seed=5)
    rng = np.random.default_rng(17)
    P[:16, 3] = 1.0 + rng.random(16) * 4.0          # e in (1, 5]
    P[16, 3] = np.nextafter(1.0, 2.0)               # the first e with 1 - e^2 < 0
    P[17, 3] = 1.0                                  # 1 - e^2 = 0: NaN like the reference's 0/0 beta
    P[18:24, 3] = -1.0 - rng.random(6) * 2.0        # e < -1: Roche or NaN
    P[24, 3] = -1.0                                 # 1 - e^2 = 0: the reference's beta is 0 / 0
    with HBLikelihood(t, f, s) as L:
        a = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P[[16, 17, 24]])
    assert np.array_equal(a, rev, equal_nan=True)
    ref = oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    assert np.isnan(ref[:17]).all() and np.isnan(a[:17]).all()
    close_logl(a, ref)
    # templates at |e| >= 1: NaN wherever the reference's are (e = 1 too, though its logL is the Roche sentinel)
    rt = oracle.light_curve_batch(t, P[[16, 17, 24]], 8)
    assert np.array_equal(np.isnan(tm), np.isnan(rt))


@pytest.mark.parametrize("n", [300, 1024, 6001])
def test_non_finite_parameter_in_each_slot(hbmi, oracle, n):
    """A NaN, +inf or -inf in any one of the 21 parameters (the C-ABI takes
    whatever the caller passes): logL against the reference's restatement --
    NaN where it is NaN, the Roche sentinel and +-inf exactly, finite values
    within 1e-10 -- on the one-wave (N = 300, 1024) and block (6001) plans."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    # not -inf in the radius-spread slots 7 / 8: a star of radius 0, whose
    # eclipse factor Norm / (pi R^2) is 0 / 0 -- the reference multiplies it
    # into every cadence where that star is behind (NaN), the kernels only into
    # overlapping ones
    cases = [(v, i) for v in (np.nan, np.inf, -np.inf) for i in range(21) if not (v == -np.inf and i in (7, 8))]
    P = np.repeat(synth.THETA_STAR[None, :], len(cases) + 1, 0)
    for r, (v, i) in enumerate(cases):
        P[r, i] = v
    with HBLikelihood(t, f, s) as L:
        ll = L.loglike(P)
    ref = oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
    assert np.array_equal(np.isnan(ll), np.isnan(ref)), np.flatnonzero(np.isnan(ll) != np.isnan(ref))
    inf = np.isinf(ref)
    assert np.array_equal(ll[inf], ref[inf]) and not np.isinf(ll[~inf]).any()
    fin = np.isfinite(ref)
    close_logl(ll[fin], ref[fin])


# ------------------------------------------------- full-size (config C4)
def test_full_size_c4_against_oracle_and_properties(hbmi, oracle):
    """W = 65 536, N = 1024 (BASELINE config C4's whole ensemble on one GPU):
    oracle on a 512-walker sample; on all walkers determinism, permutation
    equivariance, the Roche fraction, and shard independence -- the eight
    8192-walker shards a C4 rank evaluates give the full batch's values bit
    for bit (what the sharded sampler relies on)."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.dist import shard
    from hb_mcmc_amd.likelihood import HBLikelihood

    W = 65536
    t, f, s = synth.dataset(1024, oracle.light_curve)
    P = synth.walkers(W, seed=44)
    with HBLikelihood(t, f, s) as L:
        L.reserve(W)
        a = L.loglike(P)
        b = L.loglike(P)
        perm = np.random.default_rng(3).permutation(W)
        c = L.loglike(P[perm])
        parts = [L.loglike(P[lo:hi]) for lo, hi in (shard(W, r, 8) for r in range(8))]
    assert np.array_equal(a, b, equal_nan=True)
    assert np.array_equal(a[perm], c, equal_nan=True)
    assert np.array_equal(np.concatenate(parts), a, equal_nan=True)
    idx = np.arange(0, W, 128)
    ref = oracle.loglike_batch(t, f, s, P[idx], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 16)
    close_logl(a[idx], ref)
    roche = (a == -5e14)
    assert 0.02 < roche.mean() < 0.2
    bad = np.nonzero(~np.isfinite(a))[0]
    assert len(bad) <= W // 1000
    if len(bad):  # every non-finite value is the reference's own (eclipse_area's asin domain)
        close_logl(a[bad], oracle.loglike_batch(t, f, s, P[bad], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 16))


# ------------------------------------------------- full-size (config C3)
def test_full_size_c3_against_oracle(hbmi, oracle):
    """W = 4096, N = 20 000 (config C3, the block kernel): oracle on a
    128-walker sample plus every walker whose logL is not finite (the bench
    batch met one: the reference's own eclipse_area NaN), determinism."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    W, n = 4096, 20000
    t, f, s = synth.dataset(n, oracle.light_curve)
    P = synth.walkers(W, seed=1000)  # bench.py's first C3 batch (rank 0)
    with HBLikelihood(t, f, s) as L:
        assert L.eval_kernel == "hb_eval_block_kernel"
        a = L.loglike(P)
        b = L.loglike(P)
    assert np.array_equal(a, b, equal_nan=True)
    idx = np.arange(0, W, 32)
    bad = np.nonzero(~np.isfinite(a))[0]
    sel = np.union1d(idx, bad)
    ref = oracle.loglike_batch(t, f, s, P[sel], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 16)
    close_logl(a[sel], ref)
    assert len(bad) <= 4


@pytest.mark.parametrize("order", ["sorted", "shuffled", "reversed"])
def test_warm_start_paths_against_oracle(hbmi, oracle, order):
    """The one-wave kernel warm-starts Kepler from the previous cadence of a
    lane's chain (e <= 0.8, |dE| <= 0.25; hb_device.hpp hb_cadence_flux_chain).
    Cadence order decides whether neighbours are close in phase: sorted (the
    warm fast path), shuffled (large phase jumps: the reference start), reversed
    (negative steps); eccentricities straddle the 0.8 gate and reach the
    reference's unconverged regime (e > 0.85).  Templates and logL vs the
    oracle."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    n = 1024
    t, f, s = synth.dataset(n, oracle.light_curve)
    if order == "shuffled":
        p = np.random.default_rng(5).permutation(n)
        t, f, s = t[p], f[p], s[p]
    elif order == "reversed":
        t, f, s = t[::-1].copy(), f[::-1].copy(), s[::-1].copy()
    P = synth.walkers(24, seed=77, roche_frac=0.0)
    P[:, 3] = np.array([0.02, 0.1, 0.3, 0.5, 0.7, 0.79, 0.8, 0.81, 0.84, 0.88, 0.92, 0.97] * 2)
    with HBLikelihood(t, f, s) as L:
        ll = L.loglike(P)
        tm = L.light_curve(P)
    close_logl(ll, oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))
    ref = oracle.light_curve_batch(t, P, 8)
    ok = ~np.isnan(ref).any(1)
    tol = lc_tol(P[:, 3], ref)
    assert (np.abs(tm - ref)[ok] <= tol[ok]).all()


@pytest.mark.parametrize("n", [1024, 1500, 3000])
def test_slow_path_full_deferred_queue(hbmi, oracle, n):
    """Times shifted by 2.5e5 days put every cadence's angle outside the fast
    reducer's domain (|x| >= 2^19 rad at P = 2.07 d), so every cadence of every
    wave is queued for the reference-order slow path: each wave's deferred
    queue fills to its capacity (64 VPT entries, with the branch-free push's
    sink entry in front of it).  One-wave (N = 1024), pair (1500) and rows
    (3000) plans; logL and templates against the oracle, and batch reversal
    bit-identical."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    t, f, s = synth.dataset(n, oracle.light_curve)
    t = t + 2.5e5
    assert (2 * np.pi * t / 10.0 ** synth.THETA_STAR[2] >= 2.0 ** 19).all()
    P = synth.walkers(64, seed=n + 3, roche_frac=0.1)
    with HBLikelihood(t, f, s) as L:
        ll = L.loglike(P)
        rev = L.loglike(P[::-1].copy())[::-1]
        tm = L.light_curve(P)
    assert np.array_equal(ll, rev, equal_nan=True)
    close_logl(ll, oracle.loglike_batch(t, f, s, P, synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8))
    ref = oracle.light_curve_batch(t, P, 8)
    ok = ~np.isnan(ref).any(1)
    tol = lc_tol(P[:, 3], ref)
    assert (np.abs(tm - ref)[ok] <= tol[ok]).all()


# ------------------------------------------------- write_lc_to_file
def test_write_lc_to_file_bytes(hbmi, tmp_path):
    """write_lc_to_file (likelihood3.c:880-941) through libhbmi.so: the light
    curve (N = 10 000 > 2048: the block kernel) computed on the GPU and printed
    with %12.5e is the reference's file byte for byte.  (A template within
    1e-12 of the reference can only print differently when a value lies within
    1e-12 of a 5-digit rounding boundary; none of these fixtures has one.)"""
    g = golden("writelc.npz")
    hbmi.write_lc_to_file.argtypes = [PD, C.c_char_p]
    for k, pv in enumerate(g["params"]):
        path = tmp_path / f"lc{k}.txt"
        pv = np.ascontiguousarray(pv)
        hbmi.write_lc_to_file(p(pv), str(path).encode())
        got, want = path.read_bytes(), g[f"file{k}"].tobytes()
        if got != want:  # report the first differing line (no byte-string diff of the whole file)
            bad = next(i for i, (a, b) in enumerate(zip(got.splitlines() + [b""], want.splitlines() + [b""]))
                       if a != b)
            pytest.fail(f"fixture {k}: line {bad} differs")


@pytest.mark.parametrize("n", [2, 3, 100, 8191, 8192, 8193, 40000, 200003])
def test_quicksort_sizes(hbmi, n):
    """quickSort drop-in (likelihood3.c:70-83) across the bitonic sorter's
    regimes: one LDS tile (n <= 8192), tiles + global merge steps beyond;
    with duplicates, +-0.0, +-inf and subnormals.  Same multiset, ascending
    (np.sort); +-0.0 may trade places as in the reference's comparisons."""
    rng = np.random.default_rng(n)
    a = rng.standard_normal(n) * 10.0 ** rng.integers(-300, 300, n)
    a[rng.integers(0, n, max(1, n // 10))] = 1.5  # duplicates
    if n > 8:
        a[:6] = [0.0, -0.0, np.inf, -np.inf, 5e-324, -5e-324]
        rng.shuffle(a)
    b = a.copy()
    hbmi.quickSort(p(b), 0, n - 1)
    ref = np.sort(a)
    assert np.array_equal(b, ref)
    # a sub-range sort leaves the rest untouched
    c = a.copy()
    lo, hi = n // 4, n - 1 - n // 4
    if hi > lo:
        hbmi.quickSort(p(c), lo, hi)
        assert np.array_equal(c[lo:hi + 1], np.sort(a[lo:hi + 1]))
        assert np.array_equal(c[:lo], a[:lo]) and np.array_equal(c[hi + 1:], a[hi + 1:])
