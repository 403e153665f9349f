"""Rank body for the sharded device-sampler GPU tests (tests/test_dsharded.py),
launched with torch.distributed.run.  Every rank runs its share of the
device-resident PT-MCMC (ShardedDeviceSampler) on the box's GPU; rank 0 saves
the final state of EVERY slot (all-gathered), the run statistics summed over
ranks and each rank's RNG streams / history, for comparison with a
single-process device run of the same configuration.

    python -m torch.distributed.run --nproc-per-node R tests/_dsharded_worker.py \\
        OUT.npz W NITER LADDER NPAST N [gloo|nccl] [x]

`x`: force the exchange path (step_begin / all-gather / step_end) even on one
rank -- with nccl that is an RCCL all-gather of world size 1.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main():
    out, W, niter, ladder, npast, n = sys.argv[1], *map(int, sys.argv[2:7])
    backend = sys.argv[7] if len(sys.argv) > 7 else "gloo"
    exchange = True if (len(sys.argv) > 8 and sys.argv[8] == "x") else None
    import numpy as np
    import torch
    import torch.distributed as dist

    from hb_mcmc_amd import synth
    from hb_mcmc_amd.dist import shard
    from hb_mcmc_amd.dsampler import ShardedDeviceSampler
    from hb_mcmc_amd.likelihood import HBLikelihood
    from hb_mcmc_amd.sampler import SlotSampler

    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist.init_process_group(backend)
    R, r = dist.get_world_size(), dist.get_rank()
    try:
        t, f, s = dataset(n, synth, HBLikelihood, local)
        L = HBLikelihood(t, f, s, device=local)
        lo, hi = shard(W, r, R)
        S = SlotSampler(niter, W, synth.THETA_STAR[2], lo, hi, run=0, npast=npast, ladder=ladder)
        with ShardedDeviceSampler(S, L, exchange=exchange) as D:
            D.init_logl()
            for it in range(niter):
                D.step(it)
            x, ll, xmap, lmap, _ = D.gather_all()
            D.download()
            _, _, cid = S.get()
            cid_all = D._gather_rows(cid.astype(np.float64), D.counts).astype(np.int64)
            arrs = S.state_arrays()
            seeds = D._gather_rows(arrs["seeds"].astype(np.float64), D.counts)
            hist = D._gather_rows(arrs["history"].reshape(S.nl, -1), D.counts)
            st = S.stats()
            sums = np.array([st[k] for k in ("acc", "DEacc", "DEtrial", "cold_acc", "nswap")], dtype=np.float64)
            tot = torch.from_numpy(sums)
            if backend == "nccl":
                tot = tot.cuda()
            dist.all_reduce(tot)
            exch = D.exchanged_doubles
        if r == 0:
            np.savez(out, x=x, logl=ll, cid=cid_all, xmap=xmap, logLmap=lmap, seeds=seeds, hist=hist,
                     sums=tot.cpu().numpy(), atrial=st["atrial"], exchanged=exch)
        S.close()
        L.close()
    finally:
        dist.destroy_process_group()


def dataset(n, synth, HBLikelihood, device):
    t = synth.cadences(n)
    with HBLikelihood(t, np.ones(n), np.ones(n), device=device) as tmp:
        truth = tmp.light_curve(synth.THETA_STAR[None, :])[0]
    s = np.full(n, 1e-3)
    return t, truth + s * synth.noise(n), s


import numpy as np  # noqa: E402

if __name__ == "__main__":
    main()
