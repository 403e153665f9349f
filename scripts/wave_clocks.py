"""Per-wave lifetimes of the C2 eval kernel (experiment build with
-DHB_WAVE_CLOCKS, loaded through HBMI_LIB): start/end shader clocks, SIMD and
CU of every wave, then per-SIMD occupancy over the kernel's span, and the
in-kernel shader clock (d s_memtime / d s_memrealtime x 100 MHz per wave,
median; after >= 2 s of back-to-back launches, MI355X_MICROARCH.md DVFS item 6).

    HBMI_LIB=.../libhbmi_clk.so python scripts/wave_clocks.py [--ncad 1024] [--walkers 4096]
"""
import argparse, ctypes as C, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from hb_mcmc_amd import _lib, synth  # noqa: E402
from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ncad", type=int, default=1024)
ap.add_argument("--walkers", type=int, default=4096)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--seconds", type=float, default=2.5, help="back-to-back launches before the sampled one")
ap.add_argument("--fused", action="store_true", help="time hb_loglik_batch_dev (the fused launch when it applies)")
a = ap.parse_args()
n, w = a.ncad, a.walkers
t = synth.cadences(n)
with HBLikelihood(t, np.ones(n), np.ones(n), device=0) as tmp:
    truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
s = np.full(n, 1e-3)
f = truth + s * synth.noise(n)
L = HBLikelihood(t, f, s, device=0)
L.reserve(w)
P = torch.from_numpy(synth.walkers(w, seed=1000)).cuda()
out = torch.empty(w, dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream()
import time  # noqa: E402
t_end = time.perf_counter() + a.seconds
k = 0
while k < a.reps or time.perf_counter() < t_end:
    for _ in range(50):
        if a.fused:
            L.loglike_dev(P, out, st)
        else:
            L.prepare_dev(P, st)
            L.evaluate_dev(w, out, 0, st)
    k += 50
    torch.cuda.synchronize()
lib = _lib.lib()
prologue = None
if a.fused and L.fused_wpb(w) > 0:  # the fused prologue's marks, wave 0 of every workgroup
    nwg = (w + L.fused_wpb(w) - 1) // L.fused_wpb(w)
    pb = (C.c_ulonglong * (16 * nwg))()
    assert lib.hb_debug_prologue_clocks(pb, nwg) == 0
    pc = np.frombuffer(pb, dtype=np.uint64).reshape(nwg, 16).astype(np.int64)
    # marks 1..12 (13, the records-combined mark, went with the round-5 prologue);
    # s_memtime is per XCD, so only differences within a workgroup are kept
    d = pc[:, 1:13] - pc[:, 0:1]
    prologue = {"workgroups": int(nwg), "marks": ["params in LDS", "records in LDS", "after last barrier",
                                                  "table waves done"] +
                                                 [f"role {r} phase 1 done" for r in range(4)] +
                                                 [f"role {r} phase 2 done" for r in range(4)],
                "mean_cycles_from_entry": [float(x) for x in d.mean(axis=0)],
                "max_cycles_from_entry": [float(x) for x in d.max(axis=0)]}
NW = 10  # words per wave (hb_kernels.hip kClkWords)
buf = (C.c_ulonglong * (NW * w))()
assert lib.hb_debug_wave_clocks(buf, w) == 0
c = np.frombuffer(buf, dtype=np.uint64).reshape(w, NW).astype(np.int64)
rt = c[:, 9] - c[:, 8]  # 100 MHz ticks
t0, t1, hw, xcc = c[:, 0], c[:, 4], c[:, 5], c[:, 6]
marks = c[:, 1:4]
if (c[:, 7] > 0).any():  # mark 3: the model loop's end, before the deferred queue
    marks = np.concatenate([c[:, 7:8], marks], axis=1)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
xid = xcc & 15
key = ((xid * 8 + se) * 16 + cu) * 4 + simd
life = t1 - t0
full = (marks > 0).all(axis=1)
ph = np.diff(np.concatenate([t0[:, None], marks, t1[:, None]], axis=1), axis=1)[full]
names = ["model pass", "keys+minmax", "select", "chi2+epilogue"]
if marks.shape[1] == 4:
    names = ["model loop", "deferred queue"] + names[1:]
res = {"phase_names": names,
       "phase_mean_cycles": [float(x) for x in ph.mean(axis=0)] if len(ph) else None,
       "waves": int(w), "life_mean": float(life.mean()), "life_min": int(life.min()), "life_max": int(life.max()),
       "life_pct": [float(x) for x in np.percentile(life, [5, 25, 50, 75, 95])],
       "launches_before_sample": int(k),
       "shader_clock_ghz_median": float(np.median((life / np.maximum(rt, 1))[rt > 100]) * 0.1),
       "shader_clock_ghz_pct": [float(x) for x in np.percentile((life / np.maximum(rt, 1))[rt > 100] * 0.1,
                                                                 [5, 25, 50, 75, 95])]}
spans, occ, order = [], [], []
for k in np.unique(key):
    m = key == k
    a0, a1 = t0[m].min(), t1[m].max()
    spans.append(a1 - a0)
    occ.append(life[m].sum() / max(1, (a1 - a0)))
    srt = np.argsort(t0[m])
    order.append(list((t1[m][srt] - a0)))
# wall-clock view (s_memrealtime, 100 MHz, one counter for the whole chip):
# the launch's span from its first wave's start to its last wave's end, and
# how the wave starts and ends spread over it
r0, r1 = c[:, 8], c[:, 9]
res["realtime_span_us"] = float((r1.max() - r0.min()) / 100.0)
res["wave_start_us_pct"] = [float(x) for x in np.percentile((r0 - r0.min()) / 100.0, [0, 50, 90, 100])]
res["wave_end_us_pct"] = [float(x) for x in np.percentile((r1 - r0.min()) / 100.0, [0, 50, 90, 100])]
res["simds"] = len(spans)
res["waves_per_simd"] = float(w / len(spans))
res["simd_span_mean"] = float(np.mean(spans))
res["simd_span_max"] = int(np.max(spans))
res["simd_mean_resident_waves"] = float(np.mean(occ))
ends = [sorted(o) for o in order if len(o) == 4]
if ends:
    res["finish_order_mean_of_4"] = [float(np.mean([e[i] for e in ends])) for i in range(4)]
starts = []
for k in np.unique(key):
    m = key == k
    starts.append(np.sort(t0[m] - t0[m].min()))
res["start_stagger_mean"] = [float(np.mean([s[i] for s in starts if len(s) > i])) for i in range(4)]
if prologue is not None:  # per workgroup: entry (prologue mark 0) to its last wave's end
    wpb = L.fused_wpb(w)
    ent = pc[:, 0]
    wg = np.arange(w) // wpb
    ends_wg = np.array([t1[wg == g].max() for g in range(len(ent))])
    starts_wg = np.array([t0[wg == g].min() for g in range(len(ent))])
    prologue["wg_entry_to_first_eval_start_mean"] = float((starts_wg - ent).mean())
    prologue["wg_entry_to_last_end_mean"] = float((ends_wg - ent).mean())
    prologue["wg_entry_to_last_end_max"] = float((ends_wg - ent).max())
res["prologue"] = prologue
print(json.dumps(res, indent=1))
L.close()
