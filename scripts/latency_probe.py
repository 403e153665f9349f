"""Small-batch latency of one loglike call: one-wave vs multi-wave (latency) plan.

Times the device-resident evaluation (hb_evaluate_dev through
HBLikelihood.loglike_dev) with HIP events, W walkers, N cadences."""
import numpy as np
import torch

from hb_mcmc_amd import synth
from hb_mcmc_amd.likelihood import HBLikelihood


def run(n, w, lat, reps=2000):
    t = synth.cadences(n)
    f = np.ones(n)
    s = np.full(n, 1e-3)
    P = torch.tensor(synth.walkers(w, seed=3), device="cuda")
    with HBLikelihood(t, f, s, latency_plan=lat) as L:
        out = torch.empty(w, dtype=torch.float64, device="cuda")
        for _ in range(50):
            L.loglike_dev(P, out)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            L.loglike_dev(P, out)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3


for n in (756, 2048):
    for w in (1, 25, 100, 256):
        a, b = run(n, w, False), run(n, w, True)
        print(f"N={n} W={w}: one-wave {a:.1f} us  latency {b:.1f} us", flush=True)
