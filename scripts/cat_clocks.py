"""Per-wave timeline of the catalog's eval launch (BASELINE config C5,
hb_eval_catalog_kernel; experiment build with -DHB_WAVE_CLOCKS loaded through
HBMI_LIB): for every walker of the last call, when its wave started and ended
(s_memrealtime, 100 MHz) and its phase marks (shader clock), grouped by the
catalog's size class -- where the launch's span goes: each class's walker
cost per cadence, the start order, and the SIMDs' occupancy at the end.

    HBMI_LIB=.../libhbmi_clkf.so python scripts/cat_clocks.py [--seconds 2.5]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from hb_mcmc_amd import _lib, synth  # noqa: E402
from hb_mcmc_amd.catalog import Catalog  # noqa: E402
from hb_mcmc_amd.hbio import load_folded_catalog  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--targets", type=int, default=256)
ap.add_argument("--walkers-per-target", type=int, default=64)
ap.add_argument("--seconds", type=float, default=2.5)
a = ap.parse_args()
# the C5 workload exactly as bench.py run_c5 builds it (one rank)
real = load_folded_catalog()[:a.targets]
rng = np.random.default_rng(20260105)
nsyn = a.targets - len(real)
ncad = np.concatenate([[len(r["t"]) for r in real], rng.integers(82, 1862, nsyn)]).astype(np.int64)
targets, thetas = [], []
for k in range(a.targets):
    n = int(ncad[k])
    if k < len(real):
        r = real[k]
        targets.append((r["t"], r["flux"], r["sigma"], r["mag"], r["magerr"]))
        th = synth.THETA_STAR.copy()
        th[2] = np.log10(r["period"])
        th[6] = np.fmod(th[6], r["period"])
        thetas.append(th)
        continue
    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n), device=0) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    s_ = np.full(n, 1e-3)
    targets.append((t, truth + s_ * synth.noise(n), s_))
    thetas.append(synth.THETA_STAR)
cat = Catalog(targets, device=0)
wpt = np.full(a.targets, a.walkers_per_target, dtype=np.int32)
W = int(wpt.sum())
P = torch.from_numpy(np.concatenate([synth.walkers(a.walkers_per_target, seed=2000 + 7919 * 0 + j, theta=th)
                                     for j, th in enumerate(thetas)])).cuda()
out = torch.empty(W, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream()
t_end = time.perf_counter() + a.seconds
while time.perf_counter() < t_end:
    for _ in range(50):
        cat.loglike_dev(P, wpt, out, st)
    torch.cuda.synchronize()
lib = _lib.lib()
NW = 10  # words per wave (hb_kernels.hip kClkWords)
buf = (C.c_ulonglong * (NW * W))()
assert lib.hb_debug_wave_clocks(buf, W) == 0
c = np.frombuffer(buf, dtype=np.uint64).reshape(W, NW).astype(np.int64)
wn = np.repeat(ncad, a.walkers_per_target)  # cadences of each walker's target
cls = np.where(wn > 1024, 5, np.ceil(np.log2(np.maximum(1, (wn + 63) // 64))).astype(int))
rt0, rt1 = c[:, 8], c[:, 9]
clk0, clk1 = c[:, 0], c[:, 4]
k0 = rt0.min()
res = {"walkers": W, "span_us": float((rt1.max() - k0) / 100.0),
       "shader_clock_ghz_median": float(np.median((clk1 - clk0) / np.maximum(rt1 - rt0, 1)) * 0.1), "classes": {}}
names = {5: "pair (N > 1024)", 4: "16/lane (513-1024)", 3: "8/lane (257-512)", 2: "4/lane (129-256)",
         1: "2/lane (65-128)", 0: "1/lane (<= 64)"}
# phases (shader cycles) of the waves that ran the whole body (Roche exits
# leave no marks): model pass, deferred queue, keys + bracket, select, chi^2
marks = np.stack([c[:, 7], c[:, 1], c[:, 2], c[:, 3]], axis=1)
full = (marks > 0).all(axis=1)
ph = np.diff(np.concatenate([clk0[:, None], marks, clk1[:, None]], axis=1), axis=1)
pnames = ["model pass", "deferred queue", "keys+bracket", "select", "chi2+epilogue"]
for q in sorted(set(cls.tolist()), reverse=True):
    m = cls == q
    mf = m & full
    life = (rt1[m] - rt0[m]) / 100.0
    res["classes"][names[q]] = {
        "walkers": int(m.sum()), "full_body": int(mf.sum()), "cadences_mean": float(wn[m].mean()),
        "start_us_pct": [float(x) for x in np.percentile((rt0[m] - k0) / 100.0, [0, 50, 100])],
        "end_us_pct": [float(x) for x in np.percentile((rt1[m] - k0) / 100.0, [0, 50, 100])],
        "life_us_mean": float(life.mean()),
        "life_ns_per_cadence": float((life * 1e3 / wn[m]).mean()),
        "phase_cycles_mean": dict(zip(pnames, [float(x) for x in ph[mf].mean(axis=0)])) if mf.any() else None}
# resident waves over the span (100 MHz ticks binned to 1 us)
edges = np.arange(0, int((rt1.max() - k0) / 100) + 2)
occ = [int(((rt0 - k0) / 100.0 <= e).sum() - ((rt1 - k0) / 100.0 <= e).sum()) for e in edges]
res["resident_waves_per_us"] = occ  # walkers (a pair's two waves counted once)
wt = np.where(cls == 5, 2, 1)  # wave slots held: a pair walker holds two
res["resident_wave_slots_per_us"] = [int((wt * (((rt0 - k0) / 100.0 <= e) & ((rt1 - k0) / 100.0 > e))).sum())
                                     for e in edges]
res["resident_wave_slots_by_class_per_4us"] = {
    names[q]: [int((wt * (cls == q) * (((rt0 - k0) / 100.0 <= e) & ((rt1 - k0) / 100.0 > e))).sum())
               for e in edges[::4]] for q in sorted(set(cls.tolist()), reverse=True)}
# the records launch (hb_prep_kernel<32>, 512 workgroups at C5): prologue marks
# of the last call, shader cycles from each workgroup's entry
nwg = (W + 31) // 32
pb = (C.c_ulonglong * (16 * nwg))()
assert lib.hb_debug_prologue_clocks(pb, nwg) == 0
pc = np.frombuffer(pb, dtype=np.uint64).reshape(nwg, 16).astype(np.int64)
pm = {1: "params in LDS", 5: "role 0 phase 1", 6: "role 1 phase 1", 7: "role 2 phase 1", 8: "role 3 phase 1",
      9: "role 0 phase 2", 10: "role 1 phase 2", 11: "role 2 phase 2", 12: "role 3 phase 2", 2: "records stored",
      3: "wave 0 done (catalog table)", 4: "wave 3 done (catalog table)"}
ok = (pc[:, [0, 1, 2, 3, 4]] > 0).all(axis=1)
res["prep"] = {"workgroups": int(ok.sum()),
               "mean_cycles_from_entry": {v: float((pc[ok, k] - pc[ok, 0]).mean()) for k, v in pm.items()},
               "max_cycles_from_entry": {v: float((pc[ok, k] - pc[ok, 0]).max()) for k, v in pm.items()},
               "entry_spread_cycles": float(pc[ok, 0].max() - pc[ok, 0].min())}
print(json.dumps(res, indent=1))
cat.close()
