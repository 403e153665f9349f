"""Per-slot phases of the device loop's ds_propose launch (experiment build
with -DHB_DS_CLOCKS loaded through HBMI_LIB): for every slot of the last
iteration, its wave's phase stamps (init with the previous iteration's swap
replay, first draws, Gaussian / differential-evolution proposal, walls,
priors, stores) by temperature decile and proposal type, the launch's span
and the replay's staging / level cycles.  (The one-launch ds_step iteration
this script also timed in round 5, profiles/r05/r05e_ds_step_clocks.json, was
measured slower and removed.)

    HBMI_LIB=.../libhbmi_dsclk.so python scripts/ds_clocks.py [--iters 120]
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
ap.add_argument("--iters", type=int, default=120)
ap.add_argument("--propose", action="store_true", help="accepted for old step files (the only mode)")
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
NW = 16
buf = (C.c_ulonglong * (NW * W))()
assert lib.hb_debug_dp_clocks(buf, W) == 0
c = np.frombuffer(buf, dtype=np.uint64).reshape(W, NW)
ck = c[:, :8].astype(np.int64)
rt0, rt1 = c[:, 8].astype(np.int64), c[:, 9].astype(np.int64)
temp = c[:, 10].copy().view(np.float64)
jt = (c[:, 11] & 0xff).astype(int)
ph = np.diff(ck, axis=1)  # 0->1 init, 1->2 first draw, 2->3 proposal, 3->4 -, 4->5 walls, 5->6 priors, 6->7 stores
names = ["init", "first draw + jscale", "proposal", "-", "walls", "priors", "alpha + stores"]
k0 = rt0.min()
life = (rt1 - rt0) / 100.0
dec = np.minimum(9, (np.argsort(np.argsort(-temp)) * 10) // W)  # 0 = hottest decile
res = {"span_us": float((rt1.max() - k0) / 100.0),
       "start_us_pct": [float(x) for x in np.percentile((rt0 - k0) / 100.0, [0, 50, 100])],
       "end_us_pct": [float(x) for x in np.percentile((rt1 - k0) / 100.0, [5, 50, 90, 99, 100])],
       "life_us_pct": [float(x) for x in np.percentile(life, [5, 50, 90, 99, 100])],
       "phase_cycles_mean": dict(zip(names, [float(x) for x in ph.mean(axis=0)])),
       "by_temperature_decile": [{"decile": int(d), "life_us_median": float(np.median(life[dec == d])),
                                  "phase_cycles_median": dict(zip(names, [float(x) for x in np.median(ph[dec == d], axis=0)]))}
                                 for d in range(10)],
       "by_type": {str(t): {"slots": int((jt == t).sum()), "life_us_median": float(np.median(life[jt == t]))}
                   for t in sorted(set(jt.tolist()))},
       "last_64": {"temp_decile_median": float(np.median(dec[np.argsort(rt1)[-64:]])),
                   "life_us_median": float(np.median(life[np.argsort(rt1)[-64:]])),
                   "start_us_median": float(np.median((rt0[np.argsort(rt1)[-64:]] - k0) / 100.0)),
                   "phase_cycles_median": dict(zip(names, [float(x) for x in
                                                            np.median(ph[np.argsort(rt1)[-64:]], axis=0)])),
                   "phase_cycles_max": dict(zip(names, [float(x) for x in ph[np.argsort(rt1)[-64:]].max(axis=0)])),
                   "temp_decile_hist": [int(x) for x in np.bincount(dec[np.argsort(rt1)[-64:]], minlength=10)]},
       "slowest_64_by_life": {"life_us_median": float(np.median(np.sort(life)[-64:])),
                              "phase_cycles_median": dict(zip(names, [float(x) for x in
                                                                       np.median(ph[np.argsort(life)[-64:]], axis=0)])),
                              "temp_decile_hist": [int(x) for x in
                                                   np.bincount(dec[np.argsort(life)[-64:]], minlength=10)]},
       "shader_clock_ghz_median": float(np.median((ck[:, 7] - ck[:, 0]) / np.maximum(rt1 - rt0, 1)) * 0.1)}
rp = c[:, 12:16].astype(np.int64)
if (rp[:, 0] > 0).any():  # the deferred-swap replay (defer builds): staging, levels, entries, levels
    m = rp[:, 0] > 0
    res["swap_replay"] = {"staging_cycles_pct": [float(x) for x in np.percentile((rp[m, 1] - rp[m, 0]), [5, 50, 95])],
                          "levels_cycles_pct": [float(x) for x in np.percentile((rp[m, 2] - rp[m, 1]), [5, 50, 95])],
                          "entries_pct": [float(x) for x in np.percentile(rp[m, 3] & 0xffffffff, [5, 50, 95, 100])],
                          "nlv": [int(x) for x in np.unique(rp[m, 3] >> 32)]}
print(json.dumps(res, indent=1))
S.close()
L.close()
