"""Why the likelihood kernel costs more inside the PT-MCMC loop than on the
bench's synthetic walkers: time hb_evaluate_dev (HIP events) on (a) the bench's
walkers, (b) the device sampler's states after K iterations (all 50-rung
ladder positions), (c) those states split into cold and hot rungs.  Prints one
JSON line.

    python scripts/eval_mix.py [--walkers 4096] [--ncad 1024] [--iters 200]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hb_mcmc_amd import synth  # noqa: E402
from hb_mcmc_amd.dsampler import DeviceSampler  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402
from hb_mcmc_amd.sampler import SlotSampler  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--walkers", type=int, default=4096)
ap.add_argument("--ncad", type=int, default=1024)
ap.add_argument("--iters", type=int, default=200)
a = ap.parse_args()
n, W = a.ncad, a.walkers
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
f = truth + s * synth.noise(n)
L = HBLikelihood(t, f, s)
L.reserve(W)
S = SlotSampler(a.iters, W, synth.THETA_STAR[2], 0, W, run=0, npast=500, ladder=1, nthreads=16)
with DeviceSampler(S, L) as D:
    D.init_logl()
    for it in range(a.iters):
        D.step(it)
    D.sync()
    xs, ls, _, _, _ = D.gather()
S.close()
xs = np.asarray(xs).reshape(W, 21)

dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream()
out = torch.empty(W, dtype=torch.float64, device=dev)


def time_eval(P, reps=20):
    Pd = torch.from_numpy(np.ascontiguousarray(P)).to(dev)
    w = P.shape[0]
    L.prepare_dev(Pd, stream)
    L.evaluate_dev(w, out, 0, stream)
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        L.prepare_dev(Pd, stream)
        e0.record(stream)
        L.evaluate_dev(w, out, 0, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms)) * 1e3


syn = synth.walkers(W, seed=1000)
rung = np.arange(W) % 50
res = {
    "walkers": W, "ncad": n, "sampler_iters": a.iters,
    "eval_us": {"bench_walkers": time_eval(syn), "sampler_states": time_eval(xs),
                "sampler_cold_rungs_0_24_x2": time_eval(np.concatenate([xs[rung < 25]] * 2)[:W]),
                "sampler_hot_rungs_25_49_x2": time_eval(np.concatenate([xs[rung >= 25]] * 2)[:W]),
                "sampler_by_e_desc": time_eval(xs[np.argsort(-xs[:, 3], kind="stable")]),
                "sampler_by_e_asc": time_eval(xs[np.argsort(xs[:, 3], kind="stable")]),
                "sampler_shuffled": time_eval(xs[np.random.default_rng(1).permutation(W)])},
    "e_mean": {"bench": float(syn[:, 3].mean()), "sampler": float(xs[:, 3].mean()),
               "sampler_e_gt_0.6": float((xs[:, 3] > 0.6).mean())},
    "e_quantiles_sampler": [float(x) for x in np.quantile(xs[:, 3], [0.1, 0.25, 0.5, 0.75, 0.9])],
    "e_gt_0.65_frac": {"bench": float((syn[:, 3] > 0.65).mean()), "sampler": float((xs[:, 3] > 0.65).mean())},
    "sampler_low_e_x": time_eval(np.concatenate([xs[xs[:, 3] < 0.6]] * 8)[:W]),
    "inc_near_90deg_frac": {"bench": float((np.abs(syn[:, 4] - np.pi / 2) < 0.2).mean()),
                            "sampler": float((np.abs(xs[:, 4] - np.pi / 2) < 0.2).mean())},
}
print(json.dumps(res), flush=True)
L.close()
