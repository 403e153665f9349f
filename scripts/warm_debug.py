"""Per-row template error vs the oracle for the warm-start parity case
(tests/test_gpu_parity.py::test_warm_start_paths_against_oracle): prints the
worst cadence of every walker row whose error exceeds the test tolerance."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from hb_mcmc_amd import synth  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402
from oracle import Oracle  # noqa: E402  (checker)

orc = Oracle()
n = 1024
for order in ["sorted", "shuffled", "reversed"]:
    t, f, s = synth.dataset(n, orc.light_curve)
    if order == "shuffled":
        p = np.random.default_rng(5).permutation(n)
        t, f, s = t[p], f[p], s[p]
    elif order == "reversed":
        t, f, s = t[::-1].copy(), f[::-1].copy(), s[::-1].copy()
    P = synth.walkers(24, seed=77, roche_frac=0.0)
    P[:, 3] = np.array([0.02, 0.1, 0.3, 0.5, 0.7, 0.79, 0.8, 0.81, 0.84, 0.88, 0.92, 0.97] * 2)
    with HBLikelihood(t, f, s) as L:
        tm = L.light_curve(P)
    ref = orc.light_curve_batch(t, P, 8)
    e = P[:, 3]
    tol = 1e-12 * np.maximum(1.0, (0.2 / (1 - e)) ** 3)[:, None]
    tol = np.maximum(tol, 1e-11 * np.abs(ref))
    for r in range(len(P)):
        d = np.abs(tm[r] - ref[r])
        bad = ~(d <= tol[r]) & ~np.isnan(ref[r])
        if bad.any():
            i = int(np.nanargmax(np.where(np.isnan(d), np.inf, d)))
            print(f"{order} row {r} e={e[r]} nbad={bad.sum()} worst i={i} t={t[i]:.9g} got={tm[r, i]!r} "
                  f"ref={ref[r, i]!r} tol={tol[r, i]:.2e} bad idx={np.nonzero(bad)[0][:12].tolist()} P={P[r].tolist()}")
print("done")
