"""Warm-start bookkeeping of the lane-chain model pass (HB_CHAIN_STATS build,
HBMI_LIB=...libhbmi_stats.so): per wave and cadence step, how often the warm
start is tried / accepted / converges, cold solves and Newton iterations."""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hb_mcmc_amd import synth, _lib
from hb_mcmc_amd.likelihood import HBLikelihood
n, w = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 4096
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
L = HBLikelihood(t, truth + s * synth.noise(n), s)
lib = _lib.lib()
buf = (C.c_ulonglong * 8)()
L.loglike(synth.walkers(w, seed=1000))
lib.hb_dbg_chain_stats(buf, 1)
L.loglike(synth.walkers(w, seed=1000))
lib.hb_dbg_chain_stats(buf, 1)
names = ["calls", "warm_tried", "warm_small", "warm_conv", "cold", "newton_its", "slow_path", "direct_sincos"]
print({k: buf[i] for i, k in enumerate(names)})
