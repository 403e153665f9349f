"""Multi-GPU PT-MCMC: the temperature slots of one sampler sharded over ranks
(SURVEY.md section 8(e)); one process per GPU, torch.distributed over RCCL.

The reference runs all NCHAINS chains of src/mcmc_wrapper2.c in one process
and evaluates every proposal with a scalar loglikelihood() call (:488-489).
Here rank r owns the contiguous slots [W*r/R, W*(r+1)/R) of the ladder
(`shard`) and per iteration

  1. draws its slots' proposals (each slot has its own RNG stream, so the
     draws do not depend on the sharding),
  2. evaluates them in ONE batched GPU launch on its own device,
  3. runs the Hastings test for its slots,
  4. all-gathers logL by slot (W doubles; RCCL on the GPU path),
  5. replays the tempering swaps (:554-563) -- every rank seeded glibc rand()
     with srand(NITER), holds the same logL vector and so reaches the same
     permutation without exchanging anything else,
  6. ships the 23-double record {x[21], logL, chain id} of every chain that
     crossed a rank boundary (all-to-all with exact splits; skipped when no
     chain crossed, which every rank can tell from the permutation),
  7. rank 0 (owner of slot 0, the cold chain) tracks the MAP point and writes
     the reference's output files; every 100 iterations the per-slot records
     are all-gathered for the chain/logL/temperature logs.

The result is the single-process sampler bit for bit (same seeds, draws,
accept decisions and files): tests/test_dist.py checks a 2-rank gloo run
against the reference's own trace.  A `loglik(P) -> logL` callable may stand
in for the GPU (the CPU tests use that); the product default is the GPU.
"""
from __future__ import annotations

import time

import numpy as np

from .sampler import REC, SlotSampler, Writer


def shard(W: int, rank: int, world: int):
    """Slots [lo, hi) of `rank` (contiguous, sizes differ by at most one)."""
    return W * rank // world, W * (rank + 1) // world


class _Comm:
    """The two collectives of the sharded step on the process group's device."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.device = (torch.device("cuda", torch.cuda.current_device()) if backend == "nccl"
                       else torch.device("cpu"))

    def gather_rows(self, local: np.ndarray, counts):
        """All-gather a variable number of rows per rank (padded to the max)."""
        torch = self.torch
        m = max(counts)
        row = local.shape[1:] if local.ndim > 1 else ()
        buf = torch.zeros((m,) + tuple(row), dtype=torch.float64, device=self.device)
        if len(local):
            buf[:len(local)] = torch.from_numpy(np.ascontiguousarray(local)).to(self.device)
        out = torch.empty((self.world * m,) + tuple(row), dtype=torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, buf, group=self.group)
        out = out.cpu().numpy()
        return np.concatenate([out[r * m:r * m + c] for r, c in enumerate(counts)])

    def all_to_all(self, send: np.ndarray, send_counts, recv_counts):
        torch = self.torch
        inp = torch.from_numpy(np.ascontiguousarray(send.reshape(-1))).to(self.device)
        out = torch.empty(int(sum(recv_counts)) * REC, dtype=torch.float64, device=self.device)
        self.dist.all_to_all_single(out, inp, [c * REC for c in recv_counts], [c * REC for c in send_counts],
                                    group=self.group)
        return out.cpu().numpy().reshape(-1, REC)

    def allreduce_sum(self, vals):
        t = self.torch.tensor(vals, dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, group=self.group)
        return t.cpu().numpy()


def run_sharded(t, flux, sigma, niter, run_id, log10_period, run=0, nchains=50, npast=500, ladder=0, nthreads=0,
                verbose=False, out_root=None, loglik=None, model=None, mag_data=None, magerr=None, group=None,
                device=None):
    """hb_mcmc_amd.sampler.run_mcmc over all ranks of `group` (torch.distributed
    must be initialised).  Every rank calls it with the same arguments; rank 0
    writes the files and its return value carries the MAP point."""
    comm = _Comm(group)
    R, r = comm.world, comm.rank
    W = int(nchains)
    if W < 2 * R:
        raise ValueError(f"nchains={W} must give every one of the {R} ranks at least two slots")
    bounds = [shard(W, q, R) for q in range(R)]
    counts = [hi - lo for lo, hi in bounds]
    lo, hi = bounds[r]
    owner = np.repeat(np.arange(R), counts)

    t = np.ascontiguousarray(t, dtype=np.float64)
    flux = np.ascontiguousarray(flux, dtype=np.float64)
    sigma = np.ascontiguousarray(sigma, dtype=np.float64)
    gpu = None
    if loglik is None or model is None:
        from .likelihood import HBLikelihood

        if device is None:
            device = comm.device.index if comm.device.type == "cuda" else 0
        gpu = HBLikelihood(t, flux, sigma, mag_data, magerr, device=device)
        gpu.reserve(max(counts))
        loglik = loglik or gpu.loglike
        model = model or (lambda p: gpu.light_curve(p[None, :])[0])

    S = SlotSampler(niter, W, log10_period, lo, hi, run=run, npast=npast, ladder=ladder, nthreads=nthreads)
    writer = None
    t_ll = t_comm = 0.0
    n_evals = 0
    n_moved = 0

    def ev(P):
        nonlocal t_ll, n_evals
        t0 = time.perf_counter()
        out = np.asarray(loglik(np.ascontiguousarray(P)), dtype=np.float64).reshape(-1)
        t_ll += time.perf_counter() - t0
        n_evals += len(P)
        return out

    try:
        x0, _, _ = S.get()
        xmap = logLmap = None
        if r == 0:
            logLmap = float(ev(x0[:1])[0])  # :342 (chain 0's state)
            xmap = x0[0].copy()
            if verbose:
                print("initial chi2 and likelihood %f \t %f" % (-2 * logLmap, logLmap))
            if out_root:
                writer = Writer(out_root, run_id, run, W)
                writer.attach(S)  # big-jump log lines of rank 0's slots (the reference logs slots 0-5)
        # whether any rank prints or writes: the periodic gathers run only then
        # (one collective here, so the flag is the same on every rank)
        report = comm.allreduce_sum([1.0 if (verbose or out_root) else 0.0])[0] > 0
        t_start = time.perf_counter()
        dst = np.arange(W)
        for it in range(int(niter)):
            y = S.propose(it)
            if it == 0:
                S.set_logl(ev(S.get()[0]))
            S.accept(it, ev(y))
            t0 = time.perf_counter()
            L_all = comm.gather_rows(S.get()[1], counts)
            t_comm += time.perf_counter() - t0
            perm, Lp = S.swap(L_all)
            src_owner = owner[perm]
            moved = src_owner != owner
            remote = None
            if moved.any():
                t0 = time.perf_counter()
                # records I send to rank q: sources I own whose destination is on q (ordered by destination)
                send_dst = [dst[moved & (src_owner == r) & (owner == q)] for q in range(R)]
                send = (S.pack(np.concatenate([perm[d] for d in send_dst]))
                        if sum(len(d) for d in send_dst) else np.empty((0, REC)))
                recv_dst = [dst[lo:hi][moved[lo:hi] & (src_owner[lo:hi] == q)] for q in range(R)]
                got = comm.all_to_all(send, [len(d) for d in send_dst], [len(d) for d in recv_dst])
                remote = np.zeros((hi - lo, REC))
                remote[np.concatenate(recv_dst).astype(np.int64) - lo] = got  # source order = destination order
                t_comm += time.perf_counter() - t0
                n_moved += int(moved.sum())
            S.apply_perm(perm, remote)
            if r == 0 and Lp[0] > logLmap:  # :565-572
                xmap = S.get()[0][0].copy()
                logLmap = float(Lp[0])
            # collectives at fixed iterations on every rank, and only when some
            # rank reports (`report`, agreed once over the ranks)
            if report and it % 1000 == 0:  # :575-589 (counters summed over ranks)
                st = S.stats()
                acc, de_acc, de_trial = comm.allreduce_sum([st["acc"], st["DEacc"], st["DEtrial"]])
                x_all = comm.gather_rows(S.get()[0], counts)
                if verbose and r == 0:
                    with np.errstate(divide="ignore", invalid="ignore"):
                        print("%d/%d logL=%.10g acc=%.3g DEacc=%.3g" % (
                            it, niter, Lp[0], np.float64(acc) / np.float64(st["atrial"]),
                            np.float64(de_acc) / np.float64(de_trial)))
                    print("Parameter values: ")
                    print("".join("%f\t" % v for v in x_all[min(10, W - 1), :5]))
            if report and it % 100 == 0:  # :593-649
                x_all = comm.gather_rows(S.get()[0], counts)
                if out_root and r == 0:
                    writer.step(it, Lp, x_all)
                    writer.light_curve(t, flux, np.asarray(model(xmap), dtype=np.float64))
                    writer.pars(False, x_all[0])
            S.end_iter(it)
        x_all = comm.gather_rows(S.get()[0], counts)
        if r == 0 and out_root:  # :655-681
            writer.light_curve(t, flux, np.asarray(model(xmap), dtype=np.float64))
            writer.pars(True, x_all[0])
        st = S.stats()
        cold_acc, evals = comm.allreduce_sum([st["cold_acc"], n_evals])
        return {"xmap": xmap, "logLmap": logLmap, "accepted": int(cold_acc), "swaps": st["nswap"],
                "seconds_total": time.perf_counter() - t_start, "seconds_loglik": t_ll, "seconds_comm": t_comm,
                "loglik_evals": int(evals), "slots": (lo, hi),
                "records_moved": n_moved}
    finally:
        if writer is not None:
            writer.close()
        S.close()
        if gpu is not None:
            gpu.close()


def run_sharded_device(t, flux, sigma, niter, run_id, log10_period, run=0, nchains=50, npast=500, ladder=0,
                       verbose=False, out_root=None, mag_data=None, magerr=None, group=None, device=None):
    """run_sharded with the device-resident loop on every rank
    (ShardedDeviceSampler): proposals, likelihood, Hastings test, history and
    the tempering swaps stay on each rank's GPU; per iteration ONE RCCL
    all-gather carries logL by slot plus the records of the chains near each
    shard's edges.  The host joins every 100 iterations for the reference's
    files (rank 0), as hb_mcmc_run_device does.  Same files, same MAP point and
    counters as the single-process sampler."""
    import torch

    from .dsampler import ShardedDeviceSampler
    from .likelihood import HBLikelihood

    comm = _Comm(group)
    R, r = comm.world, comm.rank
    W = int(nchains)
    if W < 2 * R:
        raise ValueError(f"nchains={W} must give every one of the {R} ranks at least two slots")
    lo, hi = shard(W, r, R)
    t = np.ascontiguousarray(t, dtype=np.float64)
    flux = np.ascontiguousarray(flux, dtype=np.float64)
    sigma = np.ascontiguousarray(sigma, dtype=np.float64)
    if device is None:
        device = torch.cuda.current_device()
    gpu = HBLikelihood(t, flux, sigma, mag_data, magerr, device=device)
    S = SlotSampler(niter, W, log10_period, lo, hi, run=run, npast=npast, ladder=ladder)
    writer = None
    D = None
    try:
        if r == 0 and out_root:
            writer = Writer(out_root, run_id, run, W)
            writer.attach(S)  # big-jump log lines of rank 0's slots (the reference logs slots 0-5)
        D = ShardedDeviceSampler(S, gpu, group)
        D.init_logl()
        # whether any rank prints or writes: the periodic gathers run only then
        report = comm.allreduce_sum([1.0 if (verbose or out_root) else 0.0])[0] > 0
        if r == 0 and verbose:
            _, _, _, lmap, _ = D.gather()
            print("initial chi2 and likelihood %f \t %f" % (-2 * lmap, lmap))
        t_start = time.perf_counter()
        model = (lambda p: gpu.light_curve(p[None, :])[0])
        for it in range(int(niter)):
            D.step(it)
            # collective cadence fixed by the iteration number and `report`
            # (agreed once over the ranks), so every rank calls the same
            # collectives; a run that prints and writes nothing gathers nothing
            if not report or it % 100 != 0:
                continue
            show = verbose and it % 1000 == 0
            write = bool(out_root)
            x_all, l_all, xmap, _, st = D.gather_all()
            if it % 1000 == 0:  # :575-589 (counters summed over ranks)
                acc, de_acc, de_trial = comm.allreduce_sum([st["acc"], st["DEacc"], st["DEtrial"]])
                if show and r == 0:
                    with np.errstate(divide="ignore", invalid="ignore"):
                        print("%d/%d logL=%.10g acc=%.3g DEacc=%.3g" % (
                            it, niter, l_all[0], np.float64(acc) / np.float64(st["atrial"]),
                            np.float64(de_acc) / np.float64(de_trial)))
                    print("Parameter values: ")
                    print("".join("%f\t" % v for v in x_all[min(10, W - 1), :5]))
            if write and r == 0:  # :593-649
                writer.step(it, l_all, x_all)
                writer.light_curve(t, flux, np.asarray(model(xmap), dtype=np.float64))
                writer.pars(False, x_all[0])
        x_all, _, xmap, logLmap, _ = D.gather_all()
        D.download()
        seconds = time.perf_counter() - t_start
        if r == 0 and out_root:  # :655-681
            writer.light_curve(t, flux, np.asarray(model(xmap), dtype=np.float64))
            writer.pars(True, x_all[0])
        st = S.stats()
        # a swap counts on the rank owning its lower slot (ds_swap_cone)
        cold_acc, nswap = comm.allreduce_sum([st["cold_acc"], st["nswap"]])
        return {"xmap": xmap if r == 0 else None, "logLmap": logLmap if r == 0 else None,
                "accepted": int(cold_acc), "swaps": int(nswap), "seconds_total": seconds,
                "loglik_evals": W * (int(niter) + 1), "slots": (lo, hi),
                "exchanged_doubles_per_iter": D.exchanged_doubles / max(1, int(niter))}
    finally:
        if D is not None:
            D.close()
        if writer is not None:
            writer.close()
        S.close()
        gpu.close()


def main(argv=None):
    """Multi-GPU counterpart of the hb_mcmc CLI (./HB_MCMC NITER TIC log10P run):

        python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
            -m hb_mcmc_amd.dist NITER TIC log10P run --root DIR [--chains W] ...

    One rank per GPU (LOCAL_RANK); backend nccl (RCCL) when GPUs are visible,
    gloo otherwise (--backend overrides).  Same input/output tree as hb_mcmc."""
    import argparse
    import os

    import torch
    import torch.distributed as dist

    from .hbio import read_folded_lc, read_mag_file

    ap = argparse.ArgumentParser(prog="hb_mcmc_amd.dist")
    ap.add_argument("niter", type=int)
    ap.add_argument("tic")
    ap.add_argument("log10P", type=float)
    ap.add_argument("run", type=int)
    ap.add_argument("--root", default=os.environ.get("HB_MCMC_ROOT", "."))
    ap.add_argument("--chains", type=int, default=50)
    ap.add_argument("--npast", type=int, default=500)
    ap.add_argument("--ladder", type=int, default=0)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--backend", choices=("nccl", "gloo"), default=None)
    ap.add_argument("--device-sampler", action="store_true",
                    help="device-resident loop on every rank (one all-gather per iteration)")
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = a.backend or ("nccl" if torch.cuda.device_count() > 0 else "gloo")
    if backend == "nccl" or a.device_sampler:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    dist.init_process_group(backend)
    try:
        lc = os.path.join(a.root, "data", "lightcurves", "folded_lightcurves", f"{a.tic}_new.txt")
        if not os.path.exists(lc):
            if dist.get_rank() == 0:
                print("Lightcurve datafile not found; terminating program ")  # mcmc_wrapper2.c:279-283
            return 0
        t, f, e = read_folded_lc(lc)
        mag, magerr = read_mag_file(os.path.join(a.root, "data", "magnitudes", f"{a.tic}.txt"))
        dev = local % max(1, torch.cuda.device_count())
        if a.device_sampler:
            res = run_sharded_device(t, f, e, a.niter, a.tic, a.log10P, run=a.run, nchains=a.chains, npast=a.npast,
                                     ladder=a.ladder, verbose=not a.quiet, out_root=a.root, mag_data=mag,
                                     magerr=magerr, device=dev)
            res.setdefault("seconds_loglik", -1.0)
            res.setdefault("seconds_comm", -1.0)
        else:
            res = run_sharded(t, f, e, a.niter, a.tic, a.log10P, run=a.run, nchains=a.chains, npast=a.npast,
                              ladder=a.ladder, nthreads=a.threads, verbose=not a.quiet, out_root=a.root,
                              mag_data=mag, magerr=magerr, device=dev)
        if dist.get_rank() == 0 and not a.quiet:
            print("done: %d iterations on %d ranks, %d logL evals, %.3f s total, %.3f s in the likelihood, "
                  "%.3f s in collectives; logLmap %.12g" % (a.niter, dist.get_world_size(), res["loglik_evals"],
                                                            res["seconds_total"], res["seconds_loglik"],
                                                            res["seconds_comm"], res["logLmap"]))
    finally:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
