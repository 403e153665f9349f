"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run in the development container (needs /root/reference and the binaries
``make -C oracle ref`` builds from it into oracle/_ref/):

    python tests/golden/make_golden.py

Every expected value below is produced by reference code compiled from
/root/reference/src: ``libref_lik3.so`` (likelihood3.c), the reference
sampler ``hb_mcmc_ref`` (mcmc_wrapper2.c + likelihood3.c) and the reference
Cython module ``pyHB`` (pyHB.pyx).  Inputs are the reference's own pins
(src/test_likelihoods.c:27-36, data/lightcurves/folded_lightcurves/*) plus
seeded synthetic vectors.  The fixtures are data only (inputs and outputs).
"""
from __future__ import annotations

import ctypes as C
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from hb_mcmc_amd import synth  # noqa: E402
from hb_mcmc_amd.hbio import read_folded_lc  # noqa: E402
from oracle import Reference  # noqa: E402

REF = os.environ.get("HB_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
FOLDED = os.path.join(REF, "data", "lightcurves", "folded_lightcurves")
MAG = synth.MAG_DEFAULT
MAGERR = synth.MAGERR_DEFAULT


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def random_params(g, n, theta=synth.THETA_STAR, scale=1.0):
    x = theta[None, :] + scale * synth.SIGMA_PROP[None, :] * g.standard_normal((n, 21))
    x = synth.reflect_into_box(x, 10 ** theta[2])
    x[:, 6] = np.fmod(x[:, 6], 10 ** theta[2])
    return x


def prior_draws(g, n, lc_period):
    lo, hi, _, _ = synth.prior_box(lc_period)
    x = lo[None, :] + g.random((n, 21)) * (hi - lo)[None, :]
    return x


def scalars(ref: Reference, g):
    out = {}
    lt = np.concatenate([np.linspace(3.3, 4.7, 57), [3.5, 3.7, 3.9, 4.5, 3.49999, 4.50001]])
    out["ab_in"] = lt
    out["ab_out"] = np.array([ref.get_alpha_beam(x) for x in lt])
    lm_nodes = np.log10(np.array([0.07, 0.1, 0.2, 0.26, 0.356, 0.47, 0.59, 0.655, 0.69, 0.784, 0.787, 0.87, 0.98,
                                  1.085, 1.377, 1.4, 1.65, 2.0, 2.5, 3.0, 4.4, 15.0, 40.0]))
    lm = np.concatenate([np.linspace(-1.6, 1.7, 67), lm_nodes])
    out["lm_in"] = lm
    out["getT_out"] = np.array([ref.getT(x) for x in lm])
    out["getR_out"] = np.array([ref.getR(x) for x in lm])
    out["envT_out"] = np.array([ref.envelope_Temp(x) for x in lm])
    out["envR_out"] = np.array([ref.envelope_Radius(x) for x in lm])
    q = np.concatenate([10 ** np.linspace(-2, 2, 41), [1.0]])
    out["egg_in"] = q
    out["egg_out"] = np.array([ref.eggleton(x) for x in q])
    # beaming / ellipsoidal / reflection: (P[d], M1, M2, e, inc, omega0, nu, ...)
    n = 64
    P = 10 ** g.uniform(-0.5, 1.5, n)
    M1 = 10 ** g.uniform(-1, 1, n)
    M2 = 10 ** g.uniform(-1, 1, n)
    e = g.uniform(0, 0.9, n)
    inc = g.uniform(0, np.pi, n)
    om = g.uniform(-np.pi, np.pi, n) + np.where(g.random(n) < 0.5, np.pi, 0.0)
    nu = g.uniform(-np.pi, np.pi, n)
    ab = g.uniform(0.2, 2.0, n)
    R = 10 ** g.uniform(-0.5, 0.6, n)
    mu = g.uniform(0.12, 0.2, n)
    tau = g.uniform(0.3, 0.38, n)
    aref = g.uniform(0.5, 1.5, n)
    out["beam_in"] = np.stack([P, M1, M2, e, inc, om, nu, ab], 1)
    out["beam_out"] = np.array([ref.beaming(*r) for r in out["beam_in"]])
    out["ell_in"] = np.stack([P, M1, M2, e, inc, om, nu, R, 10.0 * R, mu, tau], 1)
    out["ell_out"] = np.array([ref.ellipsoidal(*r) for r in out["ell_in"]])
    out["refl_in"] = np.stack([P, M1, M2, e, inc, om, nu, R, aref], 1)
    out["refl_out"] = np.array([ref.reflection(*r) for r in out["refl_in"]])
    # eclipse: all four regimes (none / full / partial d>dc / partial d<=dc), both radius orders
    RS = 6.955e10
    rows = []
    for _ in range(96):
        r1, r2 = 10 ** g.uniform(-0.5, 0.5, 2)
        big, sm = max(r1, r2), min(r1, r2)
        dc = np.sqrt(big * big - sm * sm)
        reg = g.integers(0, 4)
        if reg == 0:
            d = (big + sm) * g.uniform(1.0, 3.0)
        elif reg == 1:
            d = (big - sm) * g.uniform(0.0, 0.999)
        elif reg == 2:
            d = dc + (big + sm - dc) * g.uniform(0.001, 0.999)
        else:
            d = (big - sm) + (dc - (big - sm)) * g.uniform(0.0, 1.0)
        sgn = -1.0 if g.random() < 0.3 else 1.0
        rows.append([r1, r2, sgn * d * RS])
    rows += [[1.0, 1.0, 0.5 * RS], [2.0, 1.0, 1.0 * RS], [1.0, 2.0, 3.0 * RS], [1.5, 0.5, 0.0]]
    out["ecl_in"] = np.array(rows)
    out["ecl_out"] = np.array([ref.eclipse_area(*r) for r in out["ecl_in"]])
    # per-walker scalars on 64 parameter vectors
    pv = np.concatenate([random_params(g, 48, scale=3.0), prior_draws(g, 16, 10 ** synth.THETA_STAR[2])])
    out["pv"] = pv
    out["radii_out"] = np.array([ref.radii_teffs(p) for p in pv])
    out["dist"] = 10 ** g.uniform(1.5, 3.5, len(pv))
    out["mags_out"] = np.array([ref.mags(p, d) for p, d in zip(pv, out["dist"])])
    out["roche_out"] = np.array([ref.roche(p) for p in pv])
    save("scalars.npz", **out)


def traj_fixture(ref: Reference, g):
    th = synth.THETA_STAR  # src/test_likelihoods.c:33-36
    times = 4 * (np.arange(1000) / 1000)  # src/test_likelihoods.c:27-30
    MS, DAY = 1.9885e33, 86400.0
    tp = np.array([10 ** th[0] * MS, 10 ** th[1] * MS, 10 ** th[2] * DAY, th[3], th[4], th[5], th[6] * DAY])
    outs = ref.traj(times, tp)
    # extra orbits: random masses (incl. M2 > M1 -> swap), eccentricities to 0.95
    ex_tp, ex_out = [], []
    t2 = np.linspace(-3.0, 9.0, 200)
    for k in range(12):
        m1, m2 = 10 ** g.uniform(-0.5, 0.7, 2) * MS
        e = [0.0, 0.05, 0.3, 0.6, 0.8, 0.95][k % 6]
        p = np.array([m1, m2, 10 ** g.uniform(0, 1) * DAY, e, g.uniform(0, np.pi), g.uniform(-np.pi, np.pi),
                      g.uniform(-2, 2) * DAY])
        ex_tp.append(p)
        ex_out.append(np.stack(ref.traj(t2, p)))
    save("traj.npz", times=times, tp=tp, d=outs[0], z1=outs[1], z2=outs[2], rr=outs[3], ff=outs[4],
         ex_times=t2, ex_tp=np.array(ex_tp), ex_out=np.array(ex_out))


def median_fixture(ref: Reference, g):
    arrs = {}
    cases = [g.normal(size=8), g.normal(size=9), g.normal(size=2), g.normal(size=3),
             np.round(g.normal(size=64), 1), np.round(g.normal(size=65), 1),  # ties
             1.0 + 1e-3 * g.normal(size=1024), 1.0 + 1e-3 * g.normal(size=883),
             np.array([0.0, -0.0, 1.0, -1.0, 0.5, 0.0]), np.full(10, 3.25),
             np.concatenate([np.full(500, 1.0), np.full(501, 2.0)])]
    for i, a in enumerate(cases):
        arrs[f"in{i}"] = a
        arrs[f"rm{i}"] = ref.remove_median(a)
        arrs[f"qs{i}"] = ref.quicksort(a)
        k, pa = ref.partition(a)
        arrs[f"pk{i}"] = np.array([k])
        arrs[f"pa{i}"] = pa
    arrs["ncases"] = np.array([len(cases)])
    save("median.npz", **arrs)


def lc_fixture(ref: Reference, g, name, t, f, s, pv, keep_templates=True):
    tm = np.array([ref.light_curve(t, p) for p in pv])
    ll = np.array([ref.loglike(t, f, s, p, MAG, MAGERR)[0] for p in pv])
    if keep_templates:
        save(name, t=t, f=f, s=s, params=pv, templates=tm, logl=ll, mag=MAG, magerr=MAGERR)
    else:
        save(name, t=t, f=f, s=s, params=pv, logl=ll, mag=MAG, magerr=MAGERR,
             tsum=tm.sum(1), tsq=(tm * tm).sum(1), thead=tm[:, :16], ttail=tm[:, -16:])


def lc_fixtures(ref: Reference, g):
    th = synth.THETA_STAR
    lcp = 10 ** th[2]
    # synthetic N=1024 (configs C2/C4 shape): truth, jittered walkers, prior draws, Roche cases
    pv = np.concatenate([th[None, :], synth.walkers(20, seed=11), random_params(g, 6, scale=3.0),
                         prior_draws(g, 5, lcp)])
    pv[:, 2] = th[2]
    t, f, s = synth.dataset(1024, ref.light_curve)
    s = s.copy()
    s[::97] = 3e-6  # exercises the sigma clamp (likelihood3.c:824-827)
    lc_fixture(ref, g, "lc_synth1024.npz", t, f, s, pv)
    # tiny odd N
    t7 = synth.cadences(7)
    f7 = ref.light_curve(t7, th) + 1e-3 * synth.noise(7, 5)
    lc_fixture(ref, g, "lc_synth7.npz", t7, f7, np.full(7, 1e-3), pv[:8])
    # N=20000 (config C3): logL + template checksums
    t20, f20, s20 = synth.dataset(20000, ref.light_curve)
    lc_fixture(ref, g, "lc_synth20000.npz", t20, f20, s20, pv[:8], keep_templates=False)
    # real targets: 231937440 (N=883) and 237957506 (N=1861), periods from periods.txt
    for tic, per in (("231937440", 5.187367), ("237957506", 2.558648)):
        t, f, e = read_folded_lc(os.path.join(FOLDED, tic))  # header N, first N rows (mcmc_wrapper2.c:260-272)
        th_t = th.copy()
        th_t[2] = np.log10(per)
        th_t[6] = 0.3 * per
        pv_t = np.concatenate([th_t[None, :], synth.walkers(23, seed=13, theta=th_t), prior_draws(g, 8, per)])
        pv_t[:, 2] = th_t[2]
        lc_fixture(ref, g, f"lc_real{tic}.npz", t, f, e, pv_t, keep_templates=(tic == "231937440"))


def limits_fixture(ref: Reference):
    class Bounds(C.Structure):
        _fields_ = [("lo", C.c_double), ("hi", C.c_double)]

    class GB(C.Structure):
        _fields_ = [("flag", C.c_int)]

    lim = (Bounds * 21)()
    lims = (Bounds * 21)()
    gp = (GB * 21)()
    ref.lib.set_limits.argtypes = [C.POINTER(Bounds), C.POINTER(Bounds), C.POINTER(GB), C.c_double]
    ref.lib.set_limits(lim, lims, gp, 3.177254)
    sig = (C.c_double * 21)()
    ref.lib.initialize_proposals.argtypes = [C.POINTER(C.c_double), C.c_void_p]
    ref.lib.initialize_proposals(sig, None)
    save("limits.npz", limited=np.array([[b.lo, b.hi] for b in lim]), limits=np.array([[b.lo, b.hi] for b in lims]),
         gauss=np.array([x.flag for x in gp]), sigma=np.array(list(sig)), lc_period=np.array([3.177254]))


def pyhb_fixture(g):
    # the reference Cython module, compiled from src/pyHB.pyx into a temporary
    # directory outside the repository and deleted once the vectors are saved
    tmp = tempfile.mkdtemp(prefix="hb_ref_pyhb_")
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "pyhb", f"PYHB_DIR={tmp}"], check=True)
        sys.path.insert(0, tmp)
        import pyHB
        _pyhb_capture(pyHB)
    finally:
        if tmp in sys.path:
            sys.path.remove(tmp)
        shutil.rmtree(tmp, ignore_errors=True)


def _pyhb_capture(pyHB):

    th = synth.THETA_STAR
    t = synth.cadences(300)
    pv = np.concatenate([th[None, :], synth.walkers(7, seed=21)])
    lc3 = np.array([pyHB.lightcurve3(t, list(p)) for p in pv])
    f = lc3[0] + 1e-3 * synth.noise(300, 3)
    errs = np.full(300, 1e-3)
    lnr = np.array([0.0, 0.05, -0.1, 0.2, -0.2, 0.0, 0.01, -0.01])
    like = np.array([pyHB.likelihood(t, f, errs, list(p) + [r]) for p, r in zip(pv, lnr)])
    mags = np.array([pyHB.calc_mags(list(p) + [0.0], 300.0) for p in pv])
    radii = np.array([pyHB.calc_radii_and_Teffs(list(p)) for p in pv])
    lm = np.linspace(-1.4, 1.6, 31)
    gr = np.array([[pyHB.getR(x), pyHB.getT(x), pyHB.envelope_Temp(x), pyHB.envelope_Radius(x)] for x in lm])
    rl = np.array([[pyHB.test_roche_lobe(list(p) + [0.0]), pyHB.test_roche_lobe(list(p) + [0.0], "Eggleton")]
                   for p in pv])
    sp3 = np.array([[lo, hi] for lo, hi in zip(pyHB.sp3.mins, pyHB.sp3.maxs)])
    sp2 = np.array([[lo, hi] for lo, hi in zip(pyHB.sp2.mins, pyHB.sp2.maxs)])
    save("pyhb.npz", t=t, params=pv, lc3=lc3, f=f, errs=errs, lnr=lnr, like=like, mags=mags, radii=radii,
         lm=lm, getR_getT_envT_envR=gr, roche=rl, sp3=sp3, sp2=sp2,
         sp3_names=np.array(pyHB.sp3.names), sp2_names=np.array(pyHB.sp2.names))


def sampler_fixture():
    """Reference PT-MCMC trace: ./HB_MCMC 1200 127079833 0.5021 0."""
    exe = os.path.join(ROOT, "oracle", "_ref", "hb_mcmc_ref")
    tmp = tempfile.mkdtemp(prefix="hbref_")
    try:
        data = os.path.join(tmp, "data")
        for sub in ("subpars", "pars", "chains", "logL", "log", "lightcurves/mcmc_lightcurves", "magnitudes",
                    "lightcurves/folded_lightcurves"):
            os.makedirs(os.path.join(data, sub), exist_ok=True)
        os.makedirs(os.path.join(tmp, "debug"), exist_ok=True)
        shutil.copy(os.path.join(FOLDED, "127079833_new.txt"),
                    os.path.join(data, "lightcurves", "folded_lightcurves", "127079833_new.txt"))
        env = dict(os.environ, HBREF_ROOT=tmp)
        r = subprocess.run([exe, "1200", "127079833", "0.5021", "0"], cwd=tmp, env=env, capture_output=True,
                           text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(r.stderr)
        suf = "127079833_gmag_OMP_0"
        chain = np.loadtxt(os.path.join(data, "chains", f"chain.{suf}.dat"))
        logl = np.loadtxt(os.path.join(data, "logL", f"logL.{suf}.dat"))
        par = np.loadtxt(os.path.join(data, "pars", f"par.{suf}.dat"))
        subpar = np.loadtxt(os.path.join(data, "subpars", f"subpar.{suf}.dat"))
        with open(os.path.join(data, "lightcurves", "mcmc_lightcurves", f"{suf}.out")) as fh:
            fh.readline()
            out = np.loadtxt(fh)
        temps = np.array([np.loadtxt(os.path.join(tmp, "debug", f"temp_{j}_log.txt")) for j in range(50)])
        lc_t, lc_f, lc_e = read_folded_lc(os.path.join(FOLDED, "127079833_new.txt"))
        files = {}
        for rel in (f"data/pars/par.{suf}.dat", f"data/subpars/subpar.{suf}.dat",
                    f"data/lightcurves/mcmc_lightcurves/{suf}.out", "debug/temp_0_log.txt", "debug/temp_49_log.txt"):
            with open(os.path.join(tmp, rel), "rb") as fh:
                files[rel] = fh.read()
        # keep the exact text of the two main outputs as byte arrays for a textual compare
        with open(os.path.join(data, "chains", f"chain.{suf}.dat"), "rb") as fh:
            chain_txt = np.frombuffer(fh.read(), dtype=np.uint8)
        with open(os.path.join(data, "logL", f"logL.{suf}.dat"), "rb") as fh:
            logl_txt = np.frombuffer(fh.read(), dtype=np.uint8)
        save("sampler_127079833.npz", niter=np.array([1200]), log10p_arg=np.array(["0.5021"]), run=np.array([0]),
             chain=chain, logl=logl, par=par, subpar=subpar, out=out, temps=temps, chain_txt=chain_txt,
             logl_txt=logl_txt, stdout=np.array([r.stdout]), lc_t=lc_t, lc_f=lc_f, lc_e=lc_e,
             file_names=np.array(list(files.keys())),
             **{f"file{i}": np.frombuffer(v, dtype=np.uint8) for i, v in enumerate(files.values())})
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def writelc_fixture(ref: Reference, g):
    """write_lc_to_file (likelihood3.c:880-941): the reference's file bytes for
    THETA_STAR and seeded draws around it (periods 0.9-12 d)."""
    pv = np.vstack([synth.THETA_STAR[None, :], random_params(g, 5, scale=1.0)])
    pv[1:, 2] = np.log10(np.array([0.9, 2.0, 3.3, 7.5, 12.0]))
    pv[1:, 6] = np.fmod(pv[1:, 6], 10 ** pv[1:, 2])
    tmp = tempfile.mkdtemp()
    try:
        files = {}
        for k, p in enumerate(pv):
            path = os.path.join(tmp, f"lc{k}.txt")
            ref.write_lc_to_file(p, path)
            files[f"file{k}"] = np.frombuffer(open(path, "rb").read(), dtype=np.uint8)
        save("writelc.npz", params=pv, **files)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not found; goldens can only be generated in the development container")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "ref"], check=True)
    ref = Reference()
    g = np.random.Generator(np.random.PCG64(20261015))
    scalars(ref, g)
    traj_fixture(ref, g)
    median_fixture(ref, g)
    lc_fixtures(ref, g)
    limits_fixture(ref)
    pyhb_fixture(g)
    sampler_fixture()
    writelc_fixture(ref, np.random.Generator(np.random.PCG64(20261016)))


def sampler_only():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "ref"], check=True)
    sampler_fixture()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "sampler":
        sampler_only()
    elif len(sys.argv) > 1 and sys.argv[1] == "writelc":
        writelc_fixture(Reference(), np.random.Generator(np.random.PCG64(20261016)))
    else:
        main()
