"""C2 batches on one stream (bench.py's timed loop) against two contexts on
two HIP streams taking alternate batches, so a batch's first workgroups start
on the CUs the previous batch's workgroups free while it drains.  Same
walkers, same kernels; logL of both schedules compared bit for bit.

    python scripts/c2_two_streams.py [--steps 400] [--rounds 3]
"""
import argparse, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from hb_mcmc_amd import synth  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=400)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
n, w = 1024, 4096
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
f = truth + s * synth.noise(n)
dev = torch.device("cuda", 0)
Ls = [HBLikelihood(t, f, s) for _ in range(2)]
for L in Ls:
    L.reserve(w)
P = [torch.from_numpy(synth.walkers(w, seed=1000 + k)).to(dev) for k in range(4)]
outs = [torch.empty(w, dtype=torch.float64, device=dev) for _ in range(4)]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]


def run(two, steps):
    for k in range(steps):
        i = k & 1 if two else 0
        Ls[i].loglike_dev(P[k % 4], outs[k % 4], streams[i])


res = {"one": [], "two": []}
for r in range(a.rounds):
    for mode in ("one", "two"):
        run(mode == "two", 50)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(mode == "two", a.steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[mode].append(dt / a.steps * 1e6)
        print(json.dumps({"round": r, "mode": mode, "us_per_step": dt / a.steps * 1e6,
                          "evals_per_s": w * a.steps / dt}), flush=True)
ref = []
for k in range(4):
    Ls[0].loglike_dev(P[k], outs[k], streams[0])
torch.cuda.synchronize()
ref = [o.cpu().numpy().copy() for o in outs]
run(True, 8)
torch.cuda.synchronize()
same = all(np.array_equal(ref[k], outs[k].cpu().numpy(), equal_nan=True) for k in range(4))
print(json.dumps({"median_us_per_step": {m: sorted(v)[len(v) // 2] for m, v in res.items()},
                  "two_stream_logl_bit_identical": bool(same)}))
