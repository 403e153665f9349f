"""Bitwise A/B of two libhbmi builds (experiment tooling, GPU).

    HBMI_LIB=lib/variants/libhbmi_X.so python scripts/ab_parity.py dump OUT.npz
    python scripts/ab_parity.py compare A.npz B.npz

`dump` evaluates a fixed battery through the library the process loads:
C2 walkers (N = 1024, W = 4096, the warm-chain path and the Roche exits),
high-e walkers (the cold path), shuffled cadences (cold path, many eclipse
lanes), odd N = 883 / 1861 real light curves, templates (mode 1) and the C5
catalog layout; `compare` reports the first difference of every array.  A
kernel change that only moves work around (deferred eclipse terms, cheaper
key handling) must compare equal bit for bit.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(out):
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.catalog import Catalog
    from hb_mcmc_amd.hbio import load_folded_catalog
    from hb_mcmc_amd.likelihood import HBLikelihood

    res = {}
    n = 1024
    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    f = truth + 1e-3 * synth.noise(n)
    s = np.full(n, 1e-3)
    P = synth.walkers(4096, seed=11)
    Phe = synth.walkers(512, seed=12)
    Phe[:, 3] = np.linspace(0.8, 0.97, 512)  # cold path (e > kWarmEmax)
    with HBLikelihood(t, f, s) as L:
        res["c2"] = L.loglike(P)
        res["c2_he"] = L.loglike(Phe)
        res["c2_tmpl"] = L.light_curve(P[:256])
    rng = np.random.default_rng(5)
    perm = rng.permutation(n)
    with HBLikelihood(t[perm], f[perm], s) as L:  # shuffled: the cold path on every walker
        res["shuf"] = L.loglike(P[:1024])
    real = load_folded_catalog()
    for r in real:
        if len(r["t"]) in (883, 1861):
            th = synth.THETA_STAR.copy()
            th[2] = np.log10(r["period"])
            th[6] = np.fmod(th[6], r["period"])
            W = synth.walkers(512, seed=13, theta=th)
            with HBLikelihood(r["t"], r["flux"], r["sigma"], r["mag"], r["magerr"]) as L:
                res[f"real{len(r['t'])}"] = L.loglike(W)
                res[f"real{len(r['t'])}_tmpl"] = L.light_curve(W[:64])
    targets, thetas = [], []
    for r in real[:60]:
        targets.append((r["t"], r["flux"], r["sigma"], r["mag"], r["magerr"]))
        th = synth.THETA_STAR.copy()
        th[2] = np.log10(r["period"])
        th[6] = np.fmod(th[6], r["period"])
        thetas.append(th)
    with Catalog(targets) as cat:
        Pc = np.concatenate([synth.walkers(64, seed=100 + k, theta=th) for k, th in enumerate(thetas)])
        res["cat"] = cat.loglike(Pc, np.full(len(targets), 64, dtype=np.int32))
    np.savez(out, **res)
    print("dumped", out, {k: v.shape for k, v in res.items()})


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint64), y.view(np.uint64))
        if same:
            print(f"{k:14s} identical ({x.size} values)")
            continue
        bad += 1
        d = np.flatnonzero(x.view(np.uint64).ravel() != y.view(np.uint64).ravel())
        rel = np.nanmax(np.abs(x.ravel()[d] - y.ravel()[d]) / np.maximum(1.0, np.abs(x.ravel()[d])))
        print(f"{k:14s} DIFFERS at {len(d)} of {x.size} (first {d[:5]}, max rel {rel:.3e})")
    print("ALL IDENTICAL" if bad == 0 else f"{bad} arrays differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if compare(sys.argv[2], sys.argv[3]) else 0)
