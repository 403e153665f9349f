"""Template error of the cold Kepler path at high eccentricity, per eval plan
(GPU through libhbmi.so vs the oracle), and the model's own conditioning.

For every cadence: err = |gpu - ref| and the conditioning scale
    cond = |d flux / d M| * 2^-52 * max(1, |M|),   M = 2 pi (t - T0) / P,
i.e. what one ulp of the mean anomaly (the reference's own rounding of
2 pi (t DAY - T0 DAY) / (P DAY), likelihood3.c:147-150) moves the template by.
d flux / d M comes from a central difference of the oracle's light curve.

Prints one JSON object: per (plan, N, order, e) the max |err|, the max
err / lc_tol (the eccentricity-scaled absolute bound of tests/test_gpu_parity.py)
and the max err / (1e-12 + cond).  Used to derive the bounds of
test_pair_plan_sizes / test_rows_plan_cold_roche_shuffled.

  python scripts/cold_err_probe.py [--no-pair] --n 2048 2049 3000 4096
(HB_NO_PAIR=1 is read once at library load: --no-pair re-runs itself in a
child process with it set.)
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def lc_tol(e):
    e = np.clip(np.asarray(e, float), 0.0, 0.999)
    return 1e-12 * np.maximum(1.0, (0.2 / (1.0 - e)) ** 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[2048, 2049, 3000, 4096])
    ap.add_argument("--e", type=float, nargs="+", default=[0.8, 0.85, 0.9])
    ap.add_argument("--walkers", type=int, default=16)
    ap.add_argument("--no-pair", action="store_true")
    a = ap.parse_args()
    if a.no_pair and os.environ.get("HB_NO_PAIR") != "1":
        env = dict(os.environ, HB_NO_PAIR="1")
        sys.exit(subprocess.call([sys.executable] + sys.argv, env=env))
    from oracle import Oracle
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.likelihood import HBLikelihood

    orc = Oracle()
    out = {"no_pair": bool(a.no_pair), "cases": []}
    for n in a.n:
        for order in ("sorted", "shuffled"):
            t, f, s = synth.dataset(n, orc.light_curve)
            if order == "shuffled":
                p = np.random.default_rng(5).permutation(n)
                t, f, s = t[p], f[p], s[p]
            for e in a.e:
                P = synth.walkers(a.walkers, seed=n + int(1000 * e), roche_frac=0.0)
                P[:, 3] = e
                with HBLikelihood(t, f, s) as L:
                    tm = L.light_curve(P)
                    kern, wpw = L.eval_kernel, L.waves_per_walker
                ref = orc.light_curve_batch(t, P, 8)
                Pd = 10.0 ** P[:, 2]
                h = 1e-6 * Pd
                dfdt = np.empty_like(ref)
                for w in range(len(P)):
                    up = orc.light_curve(t + h[w], P[w])
                    dn = orc.light_curve(t - h[w], P[w])
                    dfdt[w] = (up - dn) / (2.0 * h[w])
                M = 2.0 * np.pi * (t[None, :] - P[:, 6:7]) / Pd[:, None]
                dfdM = np.abs(dfdt) * Pd[:, None] / (2.0 * np.pi)
                cond = dfdM * 2.0 ** -52 * np.maximum(1.0, np.abs(M))
                ok = ~np.isnan(ref)
                err = np.where(ok, np.abs(tm - ref), 0.0)
                r_tol = (err / lc_tol(P[:, 3])[:, None]).max()
                r_cond = (err / (1e-12 + cond)).max()
                rel = (err / np.maximum(1.0, np.abs(ref))).max()
                out["cases"].append(dict(n=n, order=order, e=e, kernel=kern, waves=wpw,
                                         max_abs=float(err.max()), max_over_lc_tol=float(r_tol),
                                         max_over_cond=float(r_cond), max_rel=float(rel),
                                         max_template=float(np.nanmax(np.abs(ref)))))
                print(json.dumps(out["cases"][-1]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
