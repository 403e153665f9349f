"""Where the template error of one case sits (diagnosis for cold_err_probe.py):
the worst cadences of one (N, e) case with their mean anomaly, the reference
value, the GPU value, |d flux / d M| and the eval kernel.  Env knobs of the
library (HB_NO_ROWS=1: the block kernel) select the plan.

  python scripts/cold_err_where.py N E [walkers]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from oracle import Oracle  # noqa: E402
from hb_mcmc_amd import synth  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402

n, e = int(sys.argv[1]), float(sys.argv[2])
nw = int(sys.argv[3]) if len(sys.argv) > 3 else 16
orc = Oracle()
t, f, s = synth.dataset(n, orc.light_curve)
P = synth.walkers(nw, seed=n + int(1000 * e), roche_frac=0.0)
P[:, 3] = e
with HBLikelihood(t, f, s) as L:
    tm = L.light_curve(P)
    kern, wpw = L.eval_kernel, L.waves_per_walker
ref = orc.light_curve_batch(t, P, 8)
err = np.abs(tm - ref)
Pd = 10.0 ** P[:, 2]
out = {"n": n, "e": e, "kernel": kern, "waves": wpw, "env": {k: v for k, v in os.environ.items() if k.startswith("HB_")},
       "worst": []}
for flat in np.argsort(err, axis=None)[::-1][:8]:
    w, i = np.unravel_index(flat, err.shape)
    h = 1e-6 * Pd[w]
    d = (orc.light_curve(t[i:i + 1] + h, P[w])[0] - orc.light_curve(t[i:i + 1] - h, P[w])[0]) / (2 * h)
    M = 2 * np.pi * (t[i] - P[w, 6]) / Pd[w]
    out["worst"].append(dict(walker=int(w), cad=int(i), row=int(i // ((n + 255) // 256)), t=float(t[i]),
                             M=float(M), Mmod=float(np.fmod(M, 2 * np.pi)), ref=float(ref[w, i]),
                             gpu=float(tm[w, i]), err=float(err[w, i]),
                             dfdM=float(abs(d) * Pd[w] / (2 * np.pi)),
                             err_cad_mean=float(err[w].mean())))
print(json.dumps(out, indent=1))
