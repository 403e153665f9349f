"""Per-wave timeline of the device sampler's one-launch iteration (ds_step,
experiment build with -DHB_DS_CLOCKS loaded through HBMI_LIB, HB_DS_STEP=1):
for every slot of the last iteration, when its wave entered, finished the
propose stage (after the records barrier) and finished the likelihood +
Hastings test, against the slot's temperature and e.  Answers where the
launch's length comes from: the hot slots' walls, the likelihood of hot
(high-e) walkers, or the bulk.

    HB_DS_STEP=1 HBMI_LIB=.../libhbmi_dsclk.so python scripts/ds_clocks.py [--iters 120]

--propose (the default two-launch iteration, HB_DS_STEP unset): the phases of
every slot's wave in the last ds_propose launch instead (init, first draws,
Gaussian / differential-evolution proposal, walls, priors, stores), by
temperature decile and proposal type.
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
ap.add_argument("--propose", action="store_true")
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
if a.propose:
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
                       "start_us_median": float(np.median((rt0[np.argsort(rt1)[-64:]] - k0) / 100.0))},
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
    sys.exit(0)
NW = 9
buf = (C.c_ulonglong * (NW * W))()
assert lib.hb_debug_ds_clocks(buf, W) == 0
c = np.frombuffer(buf, dtype=np.uint64).reshape(W, NW)
c0, c1, c2 = (c[:, k].astype(np.int64) for k in range(3))
r0, r1, r2 = (c[:, k].astype(np.int64) for k in range(3, 6))
temp = c[:, 7].copy().view(np.float64)
ecc = c[:, 8].copy().view(np.float64)
t0 = r0.min()
prop = (r1 - r0) / 100.0  # us
ev = (r2 - r1) / 100.0
end = (r2 - t0) / 100.0
order = np.argsort(-temp, kind="stable")
hot = temp >= np.quantile(temp, 0.9)
last = np.argsort(end)[-64:]
res = {
    "span_us": float((r2.max() - t0) / 100.0),
    "start_spread_us": float((r0.max() - t0) / 100.0),
    "propose_us_pct": [float(x) for x in np.percentile(prop, [5, 50, 90, 99, 100])],
    "eval_us_pct": [float(x) for x in np.percentile(ev, [5, 50, 90, 99, 100])],
    "end_us_pct": [float(x) for x in np.percentile(end, [5, 50, 90, 99, 100])],
    "hot_decile": {"propose_us_median": float(np.median(prop[hot])), "eval_us_median": float(np.median(ev[hot])),
                   "end_us_median": float(np.median(end[hot]))},
    "rest": {"propose_us_median": float(np.median(prop[~hot])), "eval_us_median": float(np.median(ev[~hot])),
             "end_us_median": float(np.median(end[~hot]))},
    "last_64_waves": {"temp_log14_median": float(np.median(np.log(temp[last]) / np.log(1.4))),
                      "e_median": float(np.median(ecc[last])),
                      "propose_us_median": float(np.median(prop[last])),
                      "eval_us_median": float(np.median(ev[last]))},
    "shader_clock_ghz_median": float(np.median((c2 - c0) / np.maximum(r2 - r0, 1)) * 0.1),
}
print(json.dumps(res, indent=1))
S.close()
L.close()
