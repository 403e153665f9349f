"""Warm-chain bookkeeping of the C2 eval (experiment build with -DHB_CHAIN_STATS,
loaded through HBMI_LIB): per wave, chain-step calls, warm steps that stayed on
the fast path, warm fallbacks (Newton from the iterate / cold restarts), cold
starts, Newton iterations and direct sincos evaluations.

    HBMI_LIB=.../libhbmi_stats.so python scripts/chain_stats.py
"""
import ctypes as C, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hb_mcmc_amd import _lib, synth  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402

n, w = 1024, 4096
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
L = HBLikelihood(t, truth + s * synth.noise(n), s)
P = synth.walkers(w, seed=1000)
lib = _lib.lib()
buf = (C.c_ulonglong * 8)()
lib.hb_dbg_chain_stats(buf, 1)
L.loglike(P)
assert lib.hb_dbg_chain_stats(buf, 1) == 0
c = np.array(buf[:], dtype=np.float64) / w
names = ["chain calls", "warm not fine", "warm fine", "warm converged by Newton", "cold starts",
         "Newton iterations", "-", "direct sincos"]
print(json.dumps({k: round(float(v), 3) for k, v in zip(names, c) if k != "-"}, indent=1))
