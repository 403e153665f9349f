"""Sharded device loop, per-rank timing (experiment tooling, GPU).

    HB_TREE=<tree> python -m torch.distributed.run --nproc-per-node R \\
        scripts/ds_shard_profile.py OUT.json W NITER WARM [N] [serial]

Every rank runs ShardedDeviceSampler (gloo, the ranks sharing the box's GPU)
over the C4 data shape (N cadences, ladder 1), WARM untimed iterations then
NITER timed ones; rank 0 writes each rank's ms/iteration and, when the
library has it (hb_dsampler_host_times), the host split (schedule building,
waits for a schedule, kernel issue).  Wrapped in `rocprofv3 --kernel-trace
--stats`, the kernel table gives the swap kernel's share of the ranks' GPU
time -- the replicated part of the sharded loop.
HB_TREE selects the source tree (an older build's worktree for the "before"
measurement).  `serial`: the ranks take turns on the GPU (step_begin rank by
rank, the all-gather, step_end rank by rank, each followed by a sync and a
barrier), so the kernel durations are those of one rank alone on the GPU --
the ranks of a real run each have their own; the wall time then means nothing.
"""
import json
import os
import sys
import time

ROOT = os.environ.get("HB_TREE") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out, W, niter, warm = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
    serial = len(sys.argv) > 6 and sys.argv[6] == "serial"
    import numpy as np
    import torch
    import torch.distributed as dist

    from hb_mcmc_amd import synth
    from hb_mcmc_amd.dist import shard
    from hb_mcmc_amd.dsampler import ShardedDeviceSampler
    from hb_mcmc_amd.likelihood import HBLikelihood
    from hb_mcmc_amd.sampler import SlotSampler

    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    R, r = dist.get_world_size(), dist.get_rank()
    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n)) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    s = np.full(n, 1e-3)
    f = truth + s * synth.noise(n)
    L = HBLikelihood(t, f, s)
    lo, hi = shard(W, r, R)
    S = SlotSampler(warm + niter, W, synth.THETA_STAR[2], lo, hi, run=0, npast=20, ladder=1)
    import ctypes as C

    def step(D, it):
        if not serial or not D.exchange:
            D.step(it)
            if serial:
                D.sync()
            return
        n = None
        for q in range(R):
            if q == r:
                n = int(D.lib.hb_dsampler_step_begin(D._h, it, C.c_void_p(D.send.data_ptr()), D.cap))
                assert n > 0
                D.sync()
            dist.barrier()
        out = torch.empty(R * n, dtype=torch.float64)
        dist.all_gather_into_tensor(out, D.send[:n].cpu())
        with torch.cuda.stream(D.stream):
            D.recv[:R * n].copy_(out)
        for q in range(R):
            if q == r:
                assert D.lib.hb_dsampler_step_end(D._h, it, C.c_void_p(D.recv.data_ptr()), n) == 0
                D.sync()
            dist.barrier()

    with ShardedDeviceSampler(S, L) as D:
        D.init_logl()
        for it in range(warm):
            step(D, it)
        D.sync()
        dist.barrier()
        h0 = D.host_times() if hasattr(D, "host_times") else None
        t0 = time.perf_counter()
        t_step = 0.0
        for it in range(warm, warm + niter):
            ts = time.perf_counter()
            step(D, it)
            t_step += time.perf_counter() - ts
        D.sync()
        dt = time.perf_counter() - t0
        h1 = D.host_times() if hasattr(D, "host_times") else None
        rec = {"rank": r, "ms_per_iter": 1e3 * dt / niter, "host_step_ms": 1e3 * t_step / niter}
        if h0 is not None:
            rec.update({k: 1e3 * (h1[k] - h0[k]) / niter for k in ("sched_build", "sched_wait", "issue")})
            rec["threads"] = h1["threads"]
        allrec = [None] * R
        dist.all_gather_object(allrec, rec)
    if r == 0:
        res = {"tree": ROOT, "W": W, "ranks": R, "niter": niter, "warm": warm, "n": n, "serial": serial,
               "per_rank": allrec}
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps(res))
    S.close()
    L.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
