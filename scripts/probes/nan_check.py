"""Which bench walkers give non-finite logL at a given N, and does the oracle agree?"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from hb_mcmc_amd import synth
from hb_mcmc_amd.likelihood import HBLikelihood
from oracle import Oracle
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
orc = Oracle()
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
f = truth + s * synth.noise(n)
import itertools
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
P = synth.walkers(4096, seed=seed)
with HBLikelihood(t, f, s) as L:
    ll = L.loglike(P)
bad = np.where(~np.isfinite(ll))[0]
print("N", n, "non-finite walkers:", len(bad), bad[:10])
if len(bad):
    idx = bad[:8]
    ref = orc.loglike_batch(t, f, s, P[idx], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 16)
    print("gpu", ll[idx]); print("oracle", ref)
    print("e of bad walkers", P[idx, 3])
