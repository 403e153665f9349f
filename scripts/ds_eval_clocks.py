"""Per-wave phases of the device loop's likelihood + Hastings launch
(hb_eval_wave_kernel<16, true, 1, 1, false>; experiment build with
-DHB_WAVE_CLOCKS loaded through HBMI_LIB): after N iterations of the device
sampler at W = 4096, N = 1024, for every slot's wave of the last launch its
model loop, deferred queue, keys + bracket, select and chi^2 + Hastings test
(shader cycles), by kind of walker (early exit: Roche or |e| > 1; the rest
split at the median model loop), the SIMDs' finish order and the launch's
wall-clock span -- next to the same phases of the fused C2 launch
(scripts/wave_clocks.py), to see where the device loop's eval costs more.

    HBMI_LIB=hb_mcmc_amd/lib/variants/libhbmi_clkf.so python scripts/ds_eval_clocks.py [--iters 200]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hb_mcmc_amd import _lib, synth  # noqa: E402
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
lib = _lib.lib()
NW = 10  # words per wave (hb_kernels.hip kClkWords)
buf = (C.c_ulonglong * (NW * W))()
assert lib.hb_debug_wave_clocks(buf, W) == 0
c = np.frombuffer(buf, dtype=np.uint64).reshape(W, NW).astype(np.int64)
t0, t1, hw, xcc = c[:, 0], c[:, 4], c[:, 5], c[:, 6]
r0, r1 = c[:, 8], c[:, 9]
marks = np.stack([c[:, 7], c[:, 1], c[:, 2], c[:, 3]], axis=1)  # model loop end, queue applied, keys, select
full = (marks > 0).all(axis=1)
early = ~full
life = t1 - t0
ph = np.diff(np.concatenate([t0[:, None], marks, t1[:, None]], axis=1), axis=1)
names = ["model loop", "deferred queue", "keys+bracket", "select", "chi2+hastings"]
ml = ph[:, 0]
med_ml = np.median(ml[full]) if full.any() else 0
groups = {"early exit (Roche, |e| > 1)": early, "full, model loop <= median": full & (ml <= med_ml),
          "full, model loop > median": full & (ml > med_ml)}
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
key = (((xcc & 15) * 8 + se) * 16 + cu) * 4 + simd
ends = []
for k in np.unique(key):
    m = key == k
    e = np.sort(t1[m] - t0[m].min())
    if len(e) == 4:
        ends.append(e)
res = {"walkers": W, "iters": a.iters, "realtime_span_us": float((r1.max() - r0.min()) / 100.0),
       "wave_end_us_pct": [float(x) for x in np.percentile((r1 - r0.min()) / 100.0, [5, 50, 90, 100])],
       "shader_clock_ghz_median": float(np.median((life / np.maximum(r1 - r0, 1))[(r1 - r0) > 100]) * 0.1),
       "life_mean": float(life.mean()),
       "phase_mean_cycles_full": dict(zip(names, [float(x) for x in ph[full].mean(axis=0)])) if full.any() else None,
       "groups": {g: {"waves": int(m.sum()), "life_mean": float(life[m].mean()) if m.any() else None,
                      "phase_mean_cycles": (dict(zip(names, [float(x) for x in ph[m].mean(axis=0)]))
                                            if m.any() and g != "early exit (Roche, |e| > 1)" else None)}
                  for g, m in groups.items()},
       "simd_finish_order_mean_of_4": [float(np.mean([e[i] for e in ends])) for i in range(4)] if ends else None}
print(json.dumps(res, indent=1))
S.close()
L.close()
