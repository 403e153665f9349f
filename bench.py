"""bench.py -- log-likelihood evals/s of the HB light-curve path on MI355X.

Workload (BASELINE.json configs[1]): a synthetic
1024-cadence heartbeat-binary light curve, 4096 walkers per GPU.  One "step"
= one batched log-likelihood over the rank's walkers (hb_loglik_batch_dev:
ONE launch at C2, the per-walker constants computed in the prologue of the
one-wave-per-walker model/median/chi^2 kernel; two launches, constants then
that kernel, beyond 16 walkers per CU as at C4), followed,
when N > 1, by the RCCL all-gather of every walker's logL (what the tempering
swap of mcmc_wrapper2.c:554-563 needs).  Inputs are resident in HBM before the
timed region; the walker batches rotate over 4 pre-generated sets.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C4|C5]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (N > 1, no torchrun environment) starts
torch.distributed.run with N ranks as a child process before anything touches
the GPU and exits with its status; under torchrun WORLD_SIZE must equal
--gpus.  --config C4 is BASELINE config 4: 65 536 walkers sharded over 8 GPUs,
i.e. 8192 walkers per GPU (weak scaling: 8192 x N global).

Rank 0 prints ONE JSON line.  `value` = evals over all ranks / max-over-ranks
wall time of the K timed steps.  `roofline` prices the dominant kernel
(hb_eval_wave_kernel: one wave per walker at N <= 1280, 2 / 4 waves of lane rows up to 4096; else hb_eval_block_kernel) with algorithmic bytes B(N) = 24 N + 176 per eval (SURVEY.md
8(d)) over its HIP-event-timed duration; `cpu_baseline` times the reference
likelihood3.c (oracle/_ref, else the oracle port) on the host cores on a
bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from hb_mcmc_amd import synth  # noqa: E402

if __name__ == "__main__" and len(sys.argv) == 4 and sys.argv[1] == "--cpu-baseline-child":
    torch = dist = HBLikelihood = None
else:
    import torch  # noqa: E402  (import torch before libhbmi: one HIP runtime)
    import torch.distributed as dist  # noqa: E402

    from hb_mcmc_amd.likelihood import HBLikelihood  # noqa: E402

METRIC = "log-likelihood evals/sec (walkers×steps/s), 1k-cadence HB light curve"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6    # MI355X fp64 vector (spec), SURVEY.md 8(d)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process group for N > 1 (nccl = RCCL; gloo only to rehearse ranks sharing one GPU)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", choices=("C2", "C3", "C4", "C5"), default="C2",
                    help="C2: one 1k-cadence light curve, 4096 walkers per GPU (the headline); C3: 20k cadences; "
                         "C4: 1k cadences, 8192 walkers per GPU (65 536 over 8 GPUs); C5: catalog sweep of "
                         "--targets light curves (N drawn from 82..1861), --walkers-per-target each, dealt over ranks")
    ap.add_argument("--targets", type=int, default=256)
    ap.add_argument("--walkers-per-target", type=int, default=64)
    ap.add_argument("--walkers", type=int, default=None, help="walkers per GPU (default: 4096; C4: 8192)")
    ap.add_argument("--ncad", type=int, default=None, help="cadences (default: 1024; C3: 20000)")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="launch and rendezvous only: every rank all-gathers its rank id (gloo/RCCL) and rank 0 "
                         "prints n_gpus; no GPU work (tests the --gpus N launcher on a CPU host)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample length")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed back-to-back steps before the warmup steps (shader clock ramp; 0: none)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timer", choices=("hip", "torch"), default="hip",
                    help="hip: libhbmi's fence-free HIP events (hb_timer_*); torch: torch.cuda.Event")
    ap.add_argument("--kernel-samples", type=int, default=100,
                    help="steps of the kernel-timing pass after the timed region: HIP events around every "
                         "step's prep and eval launches (an event pair costs ~5 us of stream time, so the "
                         "timed steps carry none)")
    ap.add_argument("--two-stream-steps", type=int, default=200,
                    help="C2 batches through two contexts on two streams (c2_two_streams key; 0: skip)")
    ap.add_argument("--prior-steps", type=int, default=100,
                    help="C2 shape on prior-spread walkers (c2_prior_spread key; 0: skip)")
    ap.add_argument("--sampler-iters", type=int, default=100,
                    help="also time the whole PT-MCMC iteration (mcmc_wrapper2.c loop) at the workload's W and N: "
                         "device-resident sampler vs the host sampler + GPU likelihood (0 = skip)")
    ap.add_argument("--dropin-iters", type=int, default=2000,
                    help="iterations of the reference sampler relinked against libhbmi.so (dropin field; each leg "
                         "also runs a tenth as many to take the process start out of the rate; 0 = skip)")
    a = ap.parse_args()
    if a.walkers is None:
        a.walkers = 8192 if a.config == "C4" else 4096
    if a.ncad is None:
        a.ncad = 20000 if a.config == "C3" else 1024
    return a


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a) -> int:
    """`python bench.py --gpus N` outside torchrun: run N ranks through
    torch.distributed.run in a child process.  Nothing here has touched HIP
    (importing torch does not), so this process only waits for the child."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def plumbing_check(a, rank, world):
    t = torch.tensor([float(rank)], dtype=torch.float64)
    if world > 1:
        out = torch.empty(world, dtype=torch.float64)
        if a.backend == "nccl":
            t, out = t.cuda(), out.cuda()
        dist.all_gather_into_tensor(out, t)
        got = out.cpu().tolist()
    else:
        got = [0.0]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "evals/s", "n_gpus": world,
                          "plumbing": True, "ranks_seen": got, "config": {"workload": a.config}}), flush=True)


def process_group_info(a, rank, world, local, dev):
    """What the process group saw, all-gathered over it: every rank's id, its
    LOCAL_RANK, the HIP device ordinal it runs on and that device's PCI
    location, so an N > 1 line shows N ranks on N distinct devices (or, in a
    gloo rehearsal, N ranks sharing one).  Collective: every rank calls it."""
    p = torch.cuda.get_device_properties(dev)
    mine = torch.tensor([rank, local, dev.index, p.pci_domain_id, p.pci_bus_id, p.pci_device_id],
                        dtype=torch.int64)
    if world > 1:
        on = dev if a.backend == "nccl" else torch.device("cpu")
        out = torch.empty(world * mine.numel(), dtype=torch.int64, device=on)
        dist.all_gather_into_tensor(out, mine.to(on))
        rows = out.cpu().view(world, -1).tolist()
    else:
        rows = [mine.tolist()]
    ranks = [{"rank": r[0], "local_rank": r[1], "device": r[2],
              "pci": f"{r[3]:04x}:{r[4]:02x}:{r[5]:02x}"} for r in rows]
    return {"world_size": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "ranks_seen": [r["rank"] for r in ranks],
            "distinct_devices": len({r["pci"] for r in ranks}),
            "ranks": ranks, "device_name": p.name, "devices_visible": torch.cuda.device_count()}


def cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(n, 64))


def cpu_baseline_child(n, target_s):
    """Runs in a torch-free child process (no second OpenMP runtime, no HIP
    threads): the reference likelihood3.c (oracle/_ref) or the oracle port."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    impl = orc.Reference() if orc.reference_available() else orc.Oracle()
    t, f, s = synth.dataset(n, impl.light_curve)
    print(json.dumps(cpu_baseline(t, f, s, target_s)), flush=True)


def run_cpu_baseline(n, target_s):
    import subprocess
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", str(n), str(target_s)],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-400:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(t, f, s, target_s):
    """Reference likelihood3.c (oracle/_ref) or the oracle port, OpenMP over walkers."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # measurement infrastructure only (the checker)

    kind = "reference" if (orc.reference_available()
                           and os.path.exists(os.path.join(orc.REF_DIR, "libref_batch.so"))) else "port"
    impl = orc.Reference() if kind == "reference" else orc.Oracle()
    nth = cpu_threads()
    mag, err = synth.MAG_DEFAULT, synth.MAGERR_DEFAULT
    impl.loglike_batch(t, f, s, synth.walkers(nth, seed=4241), mag, err, nth)  # spin up the thread pool
    pilot = synth.walkers(8 * nth, seed=4242)
    t0 = time.perf_counter()
    impl.loglike_batch(t, f, s, pilot, mag, err, nth)
    rate = len(pilot) / (time.perf_counter() - t0)
    w = int(max(16 * nth, rate * target_s))
    sample = synth.walkers(w, seed=4243)
    t0 = time.perf_counter()
    impl.loglike_batch(t, f, s, sample, mag, err, nth)
    dt = time.perf_counter() - t0
    one = sample[: max(8, int(rate / nth * 1.0))]  # ~1 s single-thread sample
    t1 = time.perf_counter()
    impl.loglike_batch(t, f, s, one, mag, err, 1)
    dt1 = time.perf_counter() - t1
    return {"value": w / dt, "unit": "evals/s", "cores": nth, "kind": kind,
            "sample": f"{w} walkers x 1 eval, N={len(t)} cadences, {dt:.1f} s wall on {nth} threads "
                      f"(OpenMP over walkers, mcmc_wrapper2.c:383 style)",
            "value_1core": len(one) / dt1}


class _HipEvent:
    """HIP event without the system-scope release fence (include/hbmi.h hb_timer_*),
    recorded on the stream the kernels are launched on."""

    def __init__(self):
        from hb_mcmc_amd import _lib
        self._lib = _lib.lib()
        self.h = self._lib.hb_timer_create()
        if not self.h:
            raise RuntimeError("hb_timer_create failed")

    def record(self, stream):
        import ctypes as C
        self._lib.hb_timer_record(self.h, C.c_void_p(stream.cuda_stream))

    def elapsed_time(self, other):
        return float(self._lib.hb_timer_elapsed_ms(self.h, other.h))

    def __del__(self):
        if getattr(self, "h", None):
            self._lib.hb_timer_destroy(self.h)


def sampler_e2e(L, w, iters, warm=20):
    """Whole PT-MCMC iterations per second on this light curve: the device-
    resident loop (hb_dsampler: proposals, walls, priors, likelihood, Hastings,
    history, tempering swaps as kernels) and the host loop (16 threads) driving
    the same GPU likelihood.  Both are bit-identical to the reference's
    bookkeeping (tests/test_dsampler.py); 50-rung ladder repeated (W > 2000)."""
    from hb_mcmc_amd.dsampler import DeviceSampler
    from hb_mcmc_amd.sampler import SlotSampler

    logp = float(synth.THETA_STAR[2])
    out = {"walkers": w, "iters_timed": iters, "unit": "walker-steps/s (1 likelihood eval each)"}
    # (the iterations timed are 20..320 of the run, as in every round: the
    # chains' burn-in changes what an iteration costs; the shader clock is
    # already settled by the likelihood legs that run first)
    dwarm = warm
    # the device loop: three consecutive runs of `iters` iterations, the median
    # quoted (the swap schedules come from host producer threads, so a host
    # hiccup of a few ms shows up in one run of 10 ms, not in the others)
    reps = 3
    S = SlotSampler(dwarm + reps * iters, w, logp, 0, w, run=0, npast=500, ladder=1, nthreads=16)
    runs = []
    with DeviceSampler(S, L) as D:
        D.init_logl()
        for it in range(dwarm):
            D.step(it)
        D.sync()
        for r in range(reps):
            t0 = time.perf_counter()
            for it in range(dwarm + r * iters, dwarm + (r + 1) * iters):
                D.step(it)
            D.sync()
            runs.append(time.perf_counter() - t0)
        try:  # since creation: warm-up and the three runs (diagnostic only)
            ht = D.host_times()
        except Exception:  # noqa: BLE001 -- a library without the timers
            ht = None
    dt = sorted(runs)[reps // 2]
    nit = dwarm + reps * iters
    out["device_loop"] = {"ms_per_iter": dt / iters * 1e3, "value": w * iters / dt,
                          "runs_ms_per_iter": [x / iters * 1e3 for x in runs],
                          # host side per iteration: the producer threads' schedule building (summed over
                          # threads), the issuing thread's waits for a schedule, and its kernel issue
                          "host_us_per_iter": None if ht is None else {
                              "sched_build": ht["sched_build"] / nit * 1e6, "sched_wait": ht["sched_wait"] / nit * 1e6,
                              "issue": ht["issue"] / nit * 1e6, "producer_threads": ht["threads"]}}
    S.close()
    S = SlotSampler(warm + iters, w, logp, 0, w, run=0, npast=500, ladder=1, nthreads=16)
    x, _, _ = S.get()
    S.set_logl(L.loglike(x))

    def host_iter(it):
        y = S.propose(it)
        S.accept(it, L.loglike(y))
        _, ll, _ = S.get()
        perm, _ = S.swap(ll)
        S.apply_perm(perm)
        S.end_iter(it)

    for it in range(warm):
        host_iter(it)
    t0 = time.perf_counter()
    for it in range(warm, warm + iters):
        host_iter(it)
    dt = time.perf_counter() - t0
    out["host_loop_16_threads"] = {"ms_per_iter": dt / iters * 1e3, "value": w * iters / dt}
    S.close()
    return out


def sampler_e2e_sharded(L, w, iters, rank, world, warm=20):
    """Whole PT-MCMC iterations on `world` ranks (ShardedDeviceSampler): each
    rank owns w slots of a w x world ladder (weak scaling, 50-rung ladder
    repeated) and runs proposals, likelihood, Hastings test and swaps on its
    GPU with one all-gather per iteration.  Max-over-ranks wall time."""
    from hb_mcmc_amd.dist import shard
    from hb_mcmc_amd.dsampler import ShardedDeviceSampler
    from hb_mcmc_amd.sampler import SlotSampler

    W = w * world
    lo, hi = shard(W, rank, world)
    S = SlotSampler(warm + iters, W, float(synth.THETA_STAR[2]), lo, hi, run=0, npast=500, ladder=1)
    with ShardedDeviceSampler(S, L) as D:
        D.init_logl()
        for it in range(warm):
            D.step(it)
        D.sync()
        dist.barrier()
        t0 = time.perf_counter()
        for it in range(warm, warm + iters):
            D.step(it)
        D.sync()
        dist.barrier()
        dt = time.perf_counter() - t0
        exch = D.exchanged_doubles
    S.close()
    tt = torch.tensor([dt], dtype=torch.float64, device=torch.device("cuda", L.device))
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    return {"walkers": W, "walkers_per_rank": w, "ranks": world, "iters_timed": iters,
            "unit": "walker-steps/s (1 likelihood eval each), all ranks",
            "device_loop_sharded": {"ms_per_iter": dt / iters * 1e3, "value": W * iters / dt,
                                    "exchange_bytes_per_rank_per_iter": 8.0 * exch / (warm + iters)}}


def two_streams(L, t, f, s, P, w, steps, stream, dev):
    """The same batches through two contexts on two HIP streams taking
    alternate steps: consecutive batches are independent (different walker
    sets), so a batch's workgroups start on the CUs the previous batch frees
    while its last waves drain, instead of after the whole launch.  Reported
    beside the headline (which keeps one stream, the reference sampler's
    dependent-step shape), with every logL compared bit for bit."""
    L2 = HBLikelihood(t, f, s, device=dev.index)
    L2.reserve(w)
    ctx = [L, L2]
    st = [stream, torch.cuda.Stream(device=dev)]
    nb = len(P)
    outs = [torch.empty(w, dtype=torch.float64, device=dev) for _ in range(nb)]

    def run(two, k0, k1):
        for k in range(k0, k1):
            i = k & 1 if two else 0
            ctx[i].loglike_dev(P[k % nb], outs[k % nb], st[i])

    res = {}
    for mode in ("one", "two"):
        run(mode == "two", 0, 20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(mode == "two", 0, steps)
        torch.cuda.synchronize()
        res[mode] = (time.perf_counter() - t0) / steps
    ref = []
    for k in range(nb):
        L.loglike_dev(P[k], outs[k], stream)
    torch.cuda.synchronize()
    ref = [o.cpu().numpy().copy() for o in outs]
    run(True, 0, 2 * nb)
    torch.cuda.synchronize()
    same = all(np.array_equal(ref[k], outs[k].cpu().numpy(), equal_nan=True) for k in range(nb))
    L2.close()
    return {"steps": steps, "walkers": w, "unit": "evals/s",
            "one_stream": {"ms_per_step": res["one"] * 1e3, "value": w / res["one"]},
            "two_streams": {"ms_per_step": res["two"] * 1e3, "value": w / res["two"]},
            "logl_bit_identical": bool(same),
            "what": "two contexts on two streams take alternate batches (independent walker sets); not the headline"}


def computed_prior_walkers(L, w, seed, dev, stream):
    """w walkers from the set_limits box (synth.prior_walkers) conditioned on a
    light curve being computed: no Roche overflow and |e| < 1 (logL neither
    the -5e14 sentinel nor NaN), i.e. the prior-box walkers whose cost is the
    model itself (mcmc_wrapper2.c:236-252; likelihood3.c:866-869).  The filter
    is one untimed evaluation of the candidates."""
    keep, k = [], 0
    while sum(len(x) for x in keep) < w:
        cand = synth.prior_walkers(4 * w, seed=seed + 7919 * k)
        out = torch.empty(len(cand), dtype=torch.float64, device=dev)
        L.loglike_dev(torch.from_numpy(cand).to(dev), out, stream)
        lv = out.cpu().numpy()
        keep.append(cand[np.isfinite(lv) & (lv != -5e14) & (np.abs(cand[:, 3]) < 1.0)])
        k += 1
    return np.ascontiguousarray(np.concatenate(keep)[:w])


def prior_spread(L, n, w, steps, stream, dev, timer, ks=50, computed=False):
    """The headline shape (one hb_loglik_batch_dev of w walkers over n
    cadences per step) on walkers drawn from the set_limits box like the
    reference's random initial state (mcmc_wrapper2.c:236-252, synth.
    prior_walkers): the spread of e, masses and Roche overflow the sampler's
    hot rungs keep proposing, where the headline walkers sit near the truth
    (every one on the warm Kepler chains).  Reported beside the headline, not
    as `value`."""
    nb = 4
    if computed:
        L.reserve(4 * w)
        Ph = [computed_prior_walkers(L, w, 5000 + 131 * k, dev, stream) for k in range(nb)]
    else:
        Ph = [synth.prior_walkers(w, seed=3000 + k) for k in range(nb)]
    P = [torch.from_numpy(x).to(dev) for x in Ph]
    out = torch.empty(w, dtype=torch.float64, device=dev)
    for k in range(10):
        L.loglike_dev(P[k % nb], out, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        L.loglike_dev(P[k % nb], out, stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    evs = [[make_event(timer) for _ in range(2)] for _ in range(ks)]
    for k in range(ks):
        evs[k][0].record(stream)
        L.loglike_dev(P[k % nb], out, stream)
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    kms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    lv = out.cpu().numpy()
    x = Ph[(ks - 1) % nb]
    roche = lv == -5e14
    return {"walkers": w, "ncad": n, "steps": steps, "value": w * steps / wall, "unit": "evals/s",
            "ms_per_step": wall / steps * 1e3, "kernel_ms": kms, "kernel_event_samples": ks,
            "last_batch": {"roche_frac": float(roche.mean()),
                           "e_gt_0p8_not_roche_frac": float(((x[:, 3] > 0.8) & ~roche).mean()),
                           "e_gt_0p84_cold_path_frac": float(((x[:, 3] > 0.84) & ~roche).mean()),
                           "nonfinite": int((~np.isfinite(lv)).sum())},
            "walkers_from": "synth.prior_walkers: uniform over the set_limits box (mcmc_wrapper2.c:236-252), "
                            "log P fixed, T0 folded" + (
                                "; conditioned on a computed light curve (no Roche overflow, |e| < 1: "
                                "bench.computed_prior_walkers)" if computed else "")}


DROPIN_LEGS = (("dropin", "hb_mcmc_ref_hbmi", {}),
               ("dropin_memo_off", "hb_mcmc_ref_hbmi", {"HBMI_DROPIN_MEMO": "0"}),
               ("dropin_profile", "hb_mcmc_ref_hbmi", {"HBMI_DROPIN_PROFILE": "1"}),
               ("reference_cpu", "hb_mcmc_ref", {}),
               # the caller's OpenMP runtime told not to spin at its barriers: its 25
               # threads share the box's 16-core CPU share with the drop-in's leader
               ("dropin_omp_passive", "hb_mcmc_ref_hbmi", {"OMP_WAIT_POLICY": "passive"}),
               ("reference_cpu_omp_passive", "hb_mcmc_ref", {"OMP_WAIT_POLICY": "passive"}))


def dropin_workdir(tmp, g):
    """The directory tree mcmc_wrapper2.c reads and writes under HBREF_ROOT,
    with TIC 127079833's folded light curve (the trace test's input)."""
    from hb_mcmc_amd.hbio import write_folded_lc

    d = os.path.join(tmp, "data", "lightcurves", "folded_lightcurves")
    os.makedirs(d)
    write_folded_lc(os.path.join(d, "127079833_new.txt"), g["lc_t"], g["lc_f"], g["lc_e"])
    for sub in ("subpars", "pars", "chains", "logL", "log", "lightcurves/mcmc_lightcurves"):
        os.makedirs(os.path.join(tmp, "data", sub), exist_ok=True)
    os.makedirs(os.path.join(tmp, "debug"))


def dropin_rate(niter, legs=DROPIN_LEGS, short=None, ref_dir=None):
    """The literal north_star drop-in: the reference's OWN sampler
    (src/mcmc_wrapper2.c, unmodified, 25 OpenMP threads) relinked against
    libhbmi.so (`make -C oracle dropin` -> oracle/_ref/hb_mcmc_ref_hbmi), so
    every scalar loglikelihood() call (2 per chain per iteration,
    mcmc_wrapper2.c:488-489) runs through the likelihood3.h entry point on the
    GPU.  Timed on TIC 127079833's folded light curve (the trace test's input),
    next to the same sampler built with likelihood3.c (oracle/_ref/hb_mcmc_ref)
    on the host cores.  Child processes; nothing here touches HIP.

    Every leg runs twice, `short` and `niter` iterations: `iters_per_s` is the
    sampler's rate, (niter - short) / (wall(niter) - wall(short)), the same
    rule for the GPU and the CPU legs; `startup_s` is what the process spends
    outside its iterations (for the drop-in: HIP runtime start, code-object
    load, context creation, ≈ 0.35 s, profiles/r06/r06s_dropin_fixed.txt), and
    `iters_per_s_wall` = niter / wall(niter) includes it."""
    import subprocess
    import tempfile

    ref_dir = ref_dir or os.path.join(ROOT, "oracle", "_ref")  # (tests pass stand-in programs)
    exe = os.path.join(ref_dir, "hb_mcmc_ref_hbmi")
    if not os.path.exists(exe):
        return {"error": "oracle/_ref/hb_mcmc_ref_hbmi not built (make -C oracle dropin)"}
    short = max(20, niter // 10) if short is None else short
    if not 0 < short < niter:
        raise ValueError("dropin_rate: need 0 < short < niter")
    g = np.load(os.path.join(ROOT, "tests", "golden", "sampler_127079833.npz"))
    out = {"niter": niter, "niter_short": short, "chains": 50,
           "light_curve": f"TIC 127079833 folded, N = {len(g['lc_t'])}",
           "unit": "sampler iterations/s (100 scalar loglikelihood() calls each), "
                   "(niter - niter_short) / (wall(niter) - wall(niter_short))"}

    def run(path, name, n, extra):
        with tempfile.TemporaryDirectory() as tmp:
            dropin_workdir(tmp, g)
            stats_path = os.path.join(tmp, "dropin_stats.json")
            env = dict(os.environ, HBREF_ROOT=tmp, **extra)
            if name == "hb_mcmc_ref_hbmi":
                env["HBMI_DROPIN_STATS"] = stats_path  # libhbmi writes its drop-in counters at exit
            t0 = time.perf_counter()
            r = subprocess.run([path, str(n), "127079833", "0.5021", "0"], cwd=tmp, capture_output=True,
                               text=True, timeout=600, env=env)
            dt = time.perf_counter() - t0
            st = None
            if os.path.exists(stats_path):
                with open(stats_path) as fp:
                    st = json.load(fp)
        return r, dt, st

    for key, name, extra in legs:
        path = os.path.join(ref_dir, name)
        if not os.path.exists(path):
            continue
        r0, dt0, _ = run(path, name, short, extra)
        r, dt, st = run(path, name, niter, extra)
        if r0.returncode != 0 or r.returncode != 0:
            out[key] = {"error": (r0.stderr if r0.returncode else r.stderr)[-300:]}
            continue
        rate = (niter - short) / (dt - dt0) if dt > dt0 else niter / dt
        out[key] = {"iters_per_s": rate, "loglik_calls_per_s": 100.0 * rate, "iters_per_s_wall": niter / dt,
                    "wall_s": dt, "wall_short_s": dt0, "startup_s": max(0.0, dt - niter / rate)}
        if extra:
            out[key]["env"] = extra
        if st:  # per-iteration breakdown of the drop-in's GPU round trips (hb_dropin.hpp Stats), niter run
            b = max(1, st["batches"])
            st["batches_per_iter"] = st["batches"] / niter
            st["mean_batch"] = st["walkers"] / b
            st["memo_hit_frac"] = st["memo_hits"] / max(1, st["calls"])
            st["us_per_batch"] = {k[2:]: st[k] / b * 1e6 for k in ("s_combine", "s_upload", "s_launch",
                                                                   "s_download_sync")}
            st["us_wake_per_waiter"] = st["s_wake"] / max(1, st.get("waiters", st["walkers"] - st["batches"])) * 1e6
            out[key]["stats"] = st
    d, c = out.get("dropin", {}), out.get("reference_cpu", {})
    if "iters_per_s" in d and "iters_per_s" in c:
        out["speedup_vs_reference_cpu"] = d["iters_per_s"] / c["iters_per_s"]
        out["speedup_vs_reference_cpu_wall"] = d["iters_per_s_wall"] / c["iters_per_s_wall"]
    return out


SIMDS = 1024               # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md chip table)
CLOCK_HZ = 2.4e9           # max engine clock (chip table)


def counters_for(config):
    """Per-call PMC counters of this workload measured on the kernels this
    tree builds (profiles/pmc_counters.json keyed by _lib.kernel_build_id(),
    written by scripts/pmc_summary.py), or None."""
    from hb_mcmc_amd._lib import kernel_build_id
    bid = kernel_build_id()
    path = os.path.join(ROOT, "profiles", "pmc_counters.json")
    try:
        c = json.load(open(path)).get(bid, {}).get(config)
    except (OSError, ValueError):
        c = None
    return bid, c


def shader_clock_for(config):
    """The in-kernel shader clock measured on this workload (profiles/
    shader_clock.json, written from scripts/wave_clocks.py's median), or None."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "shader_clock.json"))).get(config)
    except (OSError, ValueError):
        return None


def roofline(config, kernel_ms, evals_per_call, hbm_bytes_per_call, extra):
    """The dominant kernel's roofline.  Bound: the fp64 VALU (the path is
    elementwise fp64 transcendental work + a select).  t/f/sigma
    stay L2-resident; the measured HBM traffic (`traffic`, PMC) is mostly the
    deferred eclipse queue -- 31 MB per C2 launch against the 101 MB
    algorithmic figure, DESIGN.md section 3.  achieved = counted fp64 flops per call (PMC) / the call's
    HIP-event duration (counted work: a build that removes instructions reads a
    lower frac at the same time); the VALU-issue fraction prices the counted fp64 (4
    clk per wave64 instruction) and other VALU instructions (2 clk) against
    1024 SIMDs at 2.4 GHz.  The SURVEY 8(d) algorithmic-bytes figure is kept
    as roofline.hbm.  Without counters for this kernel build the HBM figure
    is the primary one."""
    bid, c = counters_for(config)
    sec = kernel_ms * 1e-3
    hbm = {"achieved": hbm_bytes_per_call / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": hbm_bytes_per_call / sec / 1e9 / HBM_PEAK_GBS,
           "algorithmic_bytes_per_call": hbm_bytes_per_call}
    out = {}
    if c and "fp64_flop_per_call" in c:
        tf = c["fp64_flop_per_call"] / sec / 1e12
        out = {"bound": "valu", "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
               "frac": tf / FP64_PEAK_TFLOPS, "traffic": c.get("hbm_bytes_per_call"),
               "fp64_flop_per_eval_counted": c["fp64_flop_per_call"] / evals_per_call}
        if "valu_issue_cycles_per_call" in c:
            out["valu_issue_frac"] = c["valu_issue_cycles_per_call"] / (SIMDS * CLOCK_HZ * sec)
            clk = shader_clock_for(config)
            if clk:  # priced at the clock the chip held on this workload, not the 2.4 GHz peak
                out["shader_clock_ghz"] = clk["ghz"]
                out["shader_clock_source"] = clk.get("source")
                out["valu_issue_frac_at_clock"] = c["valu_issue_cycles_per_call"] / (SIMDS * clk["ghz"] * 1e9 * sec)
        out["hbm"] = hbm
        out["counters"] = {"build": bid, "source": c.get("source")}
    else:
        out = {"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": hbm["frac"], "traffic": None,
               "counters": {"build": bid, "source": None,
                            "note": "no PMC pass recorded for this kernel build (scripts/pmc_summary.py)"}}
    out.update(extra)
    return out


def settle_agreement(a, dev, world):
    """For world > 1: a function that turns this rank's "settled" into the
    group's (every rank settled), so that every rank runs the same number of
    settle chunks -- the steps hold a collective (the logL all-gather), and a
    rank that ran one chunk more than another would leave its all-gathers
    unmatched (the group then hangs at the next barrier)."""
    if world <= 1:
        return None
    flag = torch.zeros(1, dtype=torch.int32, device=dev if a.backend == "nccl" else "cpu")

    def agree(done):
        flag.fill_(0 if done else 1)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        return int(flag.item()) == 0
    return agree


def settle_clock(step, ms, drain=None, agree=None):
    """Back-to-back steps for `ms` milliseconds before the warmup steps: the
    shader clock ramps up over the first milliseconds of sustained work
    (MI355X_MICROARCH.md, DVFS item 6: measure after back-to-back launches),
    so a handful of warmup steps alone leaves the timed steps on a rising
    clock -- 38-41 us per C2 step after 5 warmup steps against 35-36 us at
    steady state on the same box (profiles/r06/r06l_*).  Untimed; the line
    reports what ran."""
    if ms <= 0:
        return {"ms": 0.0, "steps": 0}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    k = 0
    while True:
        for _ in range(16):
            step(k)
            k += 1
        if drain is not None:
            drain()
        torch.cuda.synchronize()
        done = (time.perf_counter() - t0) * 1e3 >= ms
        if agree is not None:
            done = agree(done)  # the same chunk count on every rank
        if done:
            break
    return {"ms": (time.perf_counter() - t0) * 1e3, "steps": k,
            "why": "untimed back-to-back steps before the warmup: the shader clock ramps up under sustained load"}


def make_event(kind):
    return _HipEvent() if kind == "hip" else torch.cuda.Event(enable_timing=True)


def run_c5(a, rank, world, local, dev, pg):
    """Catalog sweep (BASELINE config C5): every step evaluates all local
    targets' walkers with one hb_catalog call (one prep launch + one eval
    launch per size class).  Targets are dealt over ranks by cadence count;
    no data-path collective (independent targets)."""
    from hb_mcmc_amd.catalog import Catalog, deal_targets

    from hb_mcmc_amd.hbio import load_folded_catalog

    # targets 0..110: the reference's folded light curves (data/folded_catalog.npz)
    # with cp_data magnitudes; the rest: synthetic fill, N ~ U[82, 1861]
    real = load_folded_catalog()[:a.targets]
    rng = np.random.default_rng(20260105)
    nsyn = a.targets - len(real)
    ncad = np.concatenate([[len(r["t"]) for r in real], rng.integers(82, 1862, nsyn)]).astype(np.int64)
    owner = deal_targets(ncad, world)
    mine = [k for k in range(a.targets) if owner[k] == rank]
    targets, thetas = [], []
    for k in mine:
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
        with HBLikelihood(t, np.ones(n), np.ones(n), device=local) as tmp:
            truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
        s_ = np.full(n, 1e-3)
        targets.append((t, truth + s_ * synth.noise(n), s_))
        thetas.append(synth.THETA_STAR)
    cat = Catalog(targets, device=local)
    wpt = np.full(len(mine), a.walkers_per_target, dtype=np.int32)
    wtot = int(wpt.sum())
    nb = 4
    P = [torch.from_numpy(np.concatenate([synth.walkers(a.walkers_per_target, seed=2000 + 97 * rank + 7919 * k + j,
                                                        theta=th) for j, th in enumerate(thetas)])).to(dev)
         for k in range(nb)]
    out = torch.empty(wtot, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()
    settle = settle_clock(lambda k: cat.loglike_dev(P[k % nb], wpt, out, stream), a.settle_ms,
                          agree=settle_agreement(a, dev, world))
    for k in range(a.warmup):
        cat.loglike_dev(P[k % nb], wpt, out, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        cat.loglike_dev(P[k % nb], wpt, out, stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    ks = max(1, a.kernel_samples)  # kernel-timing pass, events around every call
    evs = [[make_event(a.timer) for _ in range(2)] for _ in range(ks)]
    for k in range(ks):
        evs[k][0].record(stream)
        cat.loglike_dev(P[k % nb], wpt, out, stream)
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    call_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    if world > 1:
        tt = torch.tensor([wall, call_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, call_ms = (float(x) for x in tt.tolist())
    bytes_step = float(sum(a.walkers_per_target * (24 * int(ncad[k]) + 176) for k in mine))
    cat.close()
    if rank == 0:
        evals = a.targets * a.walkers_per_target * a.steps
        line = {"metric": METRIC, "value": evals / wall, "unit": "evals/s", "n_gpus": world, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": wall / a.steps * 1e3, "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64",
                "data": f"{len(real)} folded light curves of the reference (data/lightcurves/folded_lightcurves, "
                        "periods.txt; magnitudes from data/color_mag/cp_data_4-21-2022.csv) + "
                        f"{nsyn} synthetic (N ~ U[82, 1861], rng 20260105, truth = test_likelihoods.c:33-36, "
                        "sigma 1e-3); walkers around the truth at each target's period",
                "config": {"workload": f"C5: catalog sweep, {a.targets} targets x {a.walkers_per_target} walkers",
                           "targets": a.targets, "walkers_per_target": a.walkers_per_target,
                           "global_walkers": a.targets * a.walkers_per_target,
                           "parallelism": f"targets dealt over {world} GPU(s) by cadence count, no collective"},
                "settle": settle,
                "roofline": roofline("C5", call_ms, float(wtot), bytes_step,
                                     {"kernel": "hb_catalog call (hb_prep_kernel + hb_eval_catalog_kernel, every "
                                                "size class in one launch), rank 0", "kernel_ms": call_ms, "kernel_event_samples": ks,
                                      "kernel_timer": a.timer})}
        if world > 1:
            line["process_group"] = pg
        print(json.dumps(line), flush=True)


def workload_label(a, n, w, world):
    if a.config == "C4":
        return (f"C4: synthetic {n}-cadence HB light curve, {w} walkers per GPU x {world} GPU(s) = {w * world} "
                f"walkers (65 536 at 8 GPUs), logL all-gathered every step")
    return f"{'C3' if n > 2048 else 'C2'}: synthetic {n}-cadence HB light curve, {w} walkers per GPU"


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}; launch N ranks for --gpus N")
    if world > 1:
        dist.init_process_group(a.backend)
    if a.plumbing_check:
        plumbing_check(a, rank, world)
        if world > 1:
            dist.destroy_process_group()
        return
    local_rank = local
    local = local % max(1, torch.cuda.device_count())  # rehearsal: several ranks may share one GPU (gloo)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = process_group_info(a, rank, world, local_rank, dev)
    if a.config == "C5":
        run_c5(a, rank, world, local, dev, pg)
        if world > 1:
            dist.destroy_process_group()
        return

    # ---- synthetic workload (resident in HBM before timing) ----
    n, w = a.ncad, a.walkers
    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n), device=local) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    s = np.full(n, 1e-3)
    f = truth + s * synth.noise(n)
    L = HBLikelihood(t, f, s, device=local)
    L.reserve(w)
    nb = 4
    P_host = [synth.walkers(w, seed=1000 + 97 * rank + k) for k in range(nb)]
    P = [torch.from_numpy(x).to(dev) for x in P_host]
    # logL and all-gather buffers alternate between steps: step k's all-gather
    # (async, on the communicator's stream) overlaps step k+1's kernels, and
    # step k+2 waits for it before it overwrites the buffer
    outs = [torch.empty(w, dtype=torch.float64, device=dev) for _ in range(2)]
    gathered = [torch.empty(world * w, dtype=torch.float64, device=dev) for _ in range(2)]
    pending = [None, None]
    stream = torch.cuda.current_stream()

    # one step = hb_loglik_batch_dev: a single fused launch (records in the
    # eval kernel's prologue) up to 16 walkers per CU, else prep + eval; the
    # kernel-timing pass times the fused kernel, or the two launches apart
    fused = L.fused_wpb(w) > 0

    def step(k, ev=None):
        b = k & 1
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None
        if ev is not None:
            ev[0].record(stream)
        if ev is None or fused:
            L.loglike_dev(P[k % nb], outs[b], stream)
            if ev is not None:
                ev[1].record(stream)
                ev[2].record(stream)
        else:
            L.prepare_dev(P[k % nb], stream)
            ev[1].record(stream)
            L.evaluate_dev(w, outs[b], 0, stream)
            ev[2].record(stream)
        if world > 1:
            pending[b] = dist.all_gather_into_tensor(gathered[b], outs[b], async_op=True)

    def drain():
        for b in range(2):
            if pending[b] is not None:
                pending[b].wait()
                pending[b] = None

    settle = settle_clock(step, a.settle_ms, drain, settle_agreement(a, dev, world))
    for k in range(a.warmup):
        step(k)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k)
    drain()  # every step's all-gather is inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    lv = outs[(a.steps - 1) & 1].cpu().numpy()
    gl = gathered[(a.steps - 1) & 1].cpu().numpy() if world > 1 else None
    # kernel durations: a separate pass after the timed region with HIP events
    # around EVERY step's launches on the stream they run on (an event pair
    # costs ~5 us of stream time, so they stay out of the timed steps)
    ks = max(1, a.kernel_samples)
    evs = [[make_event(a.timer) for _ in range(3)] for _ in range(ks)]
    for k in range(ks):
        step(k, evs[k])
    drain()
    torch.cuda.synchronize()
    timed = evs
    if fused:  # one kernel: ev[0] -> ev[1]
        eval_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in timed]))
        prep_ms = 0.0
    else:
        prep_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in timed]))
        eval_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in timed]))
    if world > 1:
        tt = torch.tensor([wall, eval_ms, prep_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, eval_ms, prep_ms = (float(x) for x in tt.tolist())
    # sanity: the reference's model itself yields NaN for a rare walker (eclipse_area's asin
    # outside its domain, likelihood3.c:353-389) -- reproduced, counted, never more than a trace
    gather_ok = None
    if world > 1:  # the last all-gather holds every rank's logL of that batch, this rank's at its offset
        assert np.array_equal(gl[rank * w:(rank + 1) * w], lv, equal_nan=True), "all-gather mismatch"
        # ... and every other rank's: each rank checks its own slice, rank 0 reports the AND
        ok = torch.tensor([1.0], dtype=torch.float64, device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        gather_ok = bool(ok.item() == 1.0)
    nonfinite = int((~np.isfinite(lv)).sum())
    assert nonfinite <= max(1, w // 100), f"{nonfinite} non-finite logL of {w}"

    e2e = None
    if world > 1 and a.sampler_iters > 0:  # every rank takes part
        e2e = sampler_e2e_sharded(L, w, a.sampler_iters, rank, world)

    if rank == 0:
        evals = world * w * a.steps
        value = evals / wall
        bytes_per_eval = 24 * n + 176
        kernel_name = L.eval_kernel
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": wall / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md 8(d): truth = test_likelihoods.c:33-36, t_i = 2P i/N, sigma 1e-3)",
            "config": {"workload": workload_label(a, n, w, world),
                       "ncad": n, "walkers_per_gpu": w, "global_walkers": world * w,
                       "parallelism": (f"walker-sharded x{world}, logL all-gather over "
                                       f"{'RCCL' if a.backend == 'nccl' else a.backend} each step, overlapped "
                                       f"with the next step's kernels") if world > 1 else "single GPU",
                       "evals_per_walker_step": 1,
                       "note": "reference sampler spends 2 evals per walker-step (mcmc_wrapper2.c:488-489)"},
            "roofline": roofline(a.config if a.config != "C2" or n <= 2048 else "C3", eval_ms, float(w),
                                 float(bytes_per_eval * w),
                                 {"kernel": kernel_name + (f" (fused: records in its prologue, {L.fused_wpb(w)} "
                                                           "walkers per workgroup)" if fused else ""),
                                  "kernel_ms": eval_ms, "prep_kernel_ms": None if fused else prep_ms,
                                  "kernel_event_samples": len(timed), "kernel_timer": a.timer,
                                  "bytes_per_eval": bytes_per_eval}),
            "kernel_only_evals_per_s": w / ((eval_ms + prep_ms) * 1e-3),
            "settle": settle,
            "nonfinite_logl_last_batch": nonfinite,
        }
        if world > 1:
            line["process_group"] = pg
            line["allgather_check"] = {"ok": gather_ok, "doubles_per_step": world * w,
                                       "what": "last timed step's gathered logL equals each rank's own, on every rank"}
        if world == 1 and a.two_stream_steps > 0:
            line["c2_two_streams"] = two_streams(L, t, f, s, P, w, a.two_stream_steps, stream, dev)
        if world == 1 and a.prior_steps > 0 and n <= 2048:
            line["c2_prior_spread"] = prior_spread(L, n, w, a.prior_steps, stream, dev, a.timer)
            line["c2_prior_spread_computed"] = prior_spread(L, n, w, a.prior_steps, stream, dev, a.timer,
                                                            computed=True)
        if world == 1 and a.sampler_iters > 0:
            line["sampler_end_to_end"] = sampler_e2e(L, w, a.sampler_iters)
        if world > 1 and e2e is not None:
            line["sampler_end_to_end"] = e2e
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = run_cpu_baseline(n, a.cpu_seconds)
        if world == 1 and a.dropin_iters > 0:
            line["dropin"] = dropin_rate(a.dropin_iters)
            if "iters_per_s" in line["dropin"].get("dropin", {}):
                line["dropin_iters_per_s"] = line["dropin"]["dropin"]["iters_per_s"]
        print(json.dumps(line), flush=True)
    L.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) == 4 and sys.argv[1] == "--cpu-baseline-child":
        cpu_baseline_child(int(sys.argv[2]), float(sys.argv[3]))
    else:
        main()
