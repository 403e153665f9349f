"""End-to-end PT-MCMC iteration rate on one GPU (the bit-exact host-driven
sampler of include/hb_sampler.h): per iteration propose (host thread pool) ->
batched likelihood (GPU, host buffers) -> accept -> tempering swaps ->
permutation -> end_iter.  Prints per-phase milliseconds per iteration.

    python scripts/sampler_rate.py [--walkers 4096] [--ncad 1024] [--iters 200] [--threads 16]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from hb_mcmc_amd import synth  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402
from hb_mcmc_amd.sampler import SlotSampler  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--walkers", type=int, default=4096)
ap.add_argument("--ncad", type=int, default=1024)
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--device", action="store_true", help="device-resident sampler (hb_dsampler_*)")
a = ap.parse_args()

n, W = a.ncad, a.walkers
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
f = truth + s * synth.noise(n)
L = HBLikelihood(t, f, s)
L.reserve(W)
S = SlotSampler(a.iters, W, synth.THETA_STAR[2], 0, W, run=0, npast=500, ladder=1, nthreads=a.threads)
if a.device:  # device-resident loop (hb_dsampler_*): host only draws the swap schedule
    from hb_mcmc_amd.dsampler import DeviceSampler

    with DeviceSampler(S, L) as D:
        D.init_logl()
        for it in range(min(20, a.iters)):  # warm-up (code objects, first launches)
            D.step(it)
        D.sync()
        t0 = time.perf_counter()
        for it in range(20, a.iters):
            D.step(it)
        D.sync()
        wall = time.perf_counter() - t0
        _, _, _, lmap, st = D.gather()
        D.download()
    k = a.iters - 20
    print(json.dumps({"mode": "device", "walkers": W, "ncad": n, "iters": k, "ms_per_iter": wall / k * 1e3,
                      "evals_per_s": W * k / wall, "logLmap": lmap, "stats": S.stats()}))
    S.close()
    L.close()
    sys.exit(0)
x, _, _ = S.get()
S.set_logl(L.loglike(x))
ph = dict(propose=0.0, loglik=0.0, accept=0.0, swap=0.0, perm=0.0, end=0.0)
t0 = time.perf_counter()
for it in range(a.iters):
    c0 = time.perf_counter()
    y = S.propose(it)
    c1 = time.perf_counter()
    ly = L.loglike(y)
    c2 = time.perf_counter()
    S.accept(it, ly)
    c3 = time.perf_counter()
    _, ll, _ = S.get()
    perm, _ = S.swap(ll)
    c4 = time.perf_counter()
    S.apply_perm(perm)
    c5 = time.perf_counter()
    S.end_iter(it)
    c6 = time.perf_counter()
    for k, d in zip(ph, (c1 - c0, c2 - c1, c3 - c2, c4 - c3, c5 - c4, c6 - c5)):
        ph[k] += d
wall = time.perf_counter() - t0
st = S.stats()
out = {"walkers": W, "ncad": n, "iters": a.iters, "threads": a.threads,
       "ms_per_iter": wall / a.iters * 1e3, "evals_per_s": W * a.iters / wall,
       "phase_ms_per_iter": {k: v / a.iters * 1e3 for k, v in ph.items()}, "stats": st}
print(json.dumps(out))
S.close()
L.close()
