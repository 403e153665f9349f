"""Catalog-sweep mode (BASELINE config C5): many independent heartbeat
targets on one GPU, and many GPUs over a catalog.

The reference handles a catalog one target at a time: one `HB_MCMC NITER TIC
log10P run` process per TIC (src/README.txt:7, mcmc_wrapper2.c:70-73), each
calling loglikelihood() per chain per step.  Here

* `Catalog` holds every target's light curve on one GPU (concatenated in HBM
  with a per-target descriptor table, include/hbmi.h hb_catalog_*), and one
  call evaluates all targets' walkers with one prep launch and ONE eval launch
  holding every cadences-per-lane class, instead of one small launch per target;
* `run_catalog` runs one PT-MCMC per target (the mcmc_wrapper2.c loop, the
  same phase API as hb_mcmc_run) in lockstep: each iteration draws every
  target's proposals, evaluates all of them in ONE catalog call, then runs each
  target's Hastings test and swaps.  Each target's swap draws come from its
  own copy of glibc's rand() sequence (srand(NITER)), so every target's run
  is exactly the run `hb_mcmc` would make for it alone;
* `python -m hb_mcmc_amd.catalog` shards a target list over ranks (one per
  GPU, targets dealt by cadence count; no collective on the data path).

Output files: target `tic` writes the reference's tree under `<root>/<tic>/`
(the reference's debug/temp_<j>_log.txt names carry no TIC id, so targets
sharing one root would collide).
"""
from __future__ import annotations

import ctypes as C
import os
import time

import numpy as np

from . import _lib
from .sampler import SlotSampler, Writer

_PD = C.POINTER(C.c_double)


def _declare(lib):
    if getattr(lib, "_hb_catalog_declared", False):
        return lib
    lib.hb_catalog_create.restype = C.c_void_p
    lib.hb_catalog_create.argtypes = [C.c_int, C.POINTER(_PD), C.POINTER(_PD), C.POINTER(_PD),
                                      C.POINTER(C.c_long), _PD, _PD, C.c_int]
    lib.hb_catalog_destroy.argtypes = [C.c_void_p]
    lib.hb_catalog_ntargets.restype = C.c_int
    lib.hb_catalog_ntargets.argtypes = [C.c_void_p]
    for nm in ("hb_catalog_loglik", "hb_catalog_loglik_dev"):
        f = getattr(lib, nm)
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.c_void_p, C.c_void_p]
    lib._hb_catalog_declared = True
    return lib


class Catalog:
    """Light curves of many targets on one GPU.

    targets: sequence of (t, flux, sigma) or (t, flux, sigma, mag_data[5], magerr[4])."""

    def __init__(self, targets, device: int = 0):
        self.lib = _declare(_lib.lib())
        K = len(targets)
        if K == 0:
            raise ValueError("empty catalog")
        arrs, mags, errs = [], [], []
        for tg in targets:
            t, f, s = (np.ascontiguousarray(x, dtype=np.float64) for x in tg[:3])
            if not (len(t) == len(f) == len(s)):
                raise ValueError("t, flux and sigma must have equal lengths")
            arrs.append((t, f, s))
            mags.append(np.asarray(tg[3], dtype=np.float64) if len(tg) > 3 and tg[3] is not None
                        else np.array([1000.0, 1, 1, 1, 1]))
            errs.append(np.asarray(tg[4], dtype=np.float64) if len(tg) > 4 and tg[4] is not None
                        else np.full(4, 1e15))
        self._keep = arrs
        self.n = np.array([len(a[0]) for a in arrs], dtype=np.int64)
        ptrs = [(_PD * K)(*[a[i].ctypes.data_as(_PD) for a in arrs]) for i in range(3)]
        nn = (C.c_long * K)(*[int(x) for x in self.n])
        m5 = np.ascontiguousarray(np.concatenate(mags))
        e4 = np.ascontiguousarray(np.concatenate(errs))
        self._h = self.lib.hb_catalog_create(K, ptrs[0], ptrs[1], ptrs[2], nn, m5.ctypes.data_as(_PD),
                                             e4.ctypes.data_as(_PD), int(device))
        if not self._h:
            raise _lib.HBMIError("hb_catalog_create: " + _lib.last_error())
        self.ntargets = K
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hb_catalog_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @staticmethod
    def _walkers(walkers, K):
        w = np.ascontiguousarray(walkers, dtype=np.int32)
        if w.shape != (K,) or (w < 0).any():
            raise ValueError(f"walkers must be {K} non-negative counts")
        return w

    def loglike(self, params, walkers) -> np.ndarray:
        """params: (sum walkers) x 21, target 0's rows first; returns logL per row."""
        w = self._walkers(walkers, self.ntargets)
        P = np.ascontiguousarray(params, dtype=np.float64).reshape(-1, 21)
        if P.shape[0] != int(w.sum()):
            raise ValueError("params rows must equal the total walker count")
        out = np.empty(P.shape[0])
        _lib.check(self.lib.hb_catalog_loglik(self._h, P.ctypes.data_as(_PD), w.ctypes.data_as(C.POINTER(C.c_int)),
                                              out.ctypes.data_as(_PD), None), "hb_catalog_loglik")
        return out

    def loglike_dev(self, params_dev, walkers, out_dev, stream=None):
        """Device tensors (torch float64 on this GPU): params_dev (sum walkers) x 21 -> out_dev."""
        import torch
        w = self._walkers(walkers, self.ntargets)
        if params_dev.shape[0] != int(w.sum()) or out_dev.numel() != params_dev.shape[0]:
            raise ValueError("params rows and outputs must equal the total walker count")
        for x in (params_dev, out_dev):
            if not (x.is_cuda and x.dtype == torch.float64 and x.is_contiguous()):
                raise ValueError("device buffers must be contiguous float64 GPU tensors")
        s = stream if stream is not None else torch.cuda.current_stream()
        _lib.check(self.lib.hb_catalog_loglik_dev(self._h, C.c_void_p(params_dev.data_ptr()),
                                                  w.ctypes.data_as(C.POINTER(C.c_int)),
                                                  C.c_void_p(out_dev.data_ptr()), C.c_void_p(s.cuda_stream)),
                   "hb_catalog_loglik_dev")


def run_catalog(targets, niter, run_ids, log10_periods, run=0, nchains=50, npast=500, ladder=0, nthreads=0,
                out_root=None, device=0, loglik_multi=None, model=None, verbose=False):
    """One PT-MCMC per target, in lockstep, one batched catalog likelihood per step.

    targets: as for Catalog; run_ids / log10_periods: one per target.
    loglik_multi(P, walkers) -> logL may replace the GPU catalog (tests);
    model(k, params) -> model light curve of target k (for the .out files;
    default: the GPU).  Returns one result dict per target, like run_mcmc."""
    K = len(targets)
    if len(run_ids) != K or len(log10_periods) != K:
        raise ValueError("one run id and one log10 period per target")
    W = int(nchains)
    gpu_cat, gpu_lcs = None, {}
    if loglik_multi is None:
        gpu_cat = Catalog(targets, device=device)
        loglik_multi = gpu_cat.loglike
    if model is None and out_root:
        from .likelihood import HBLikelihood

        def model(k, p):
            if k not in gpu_lcs:
                t, f, s = targets[k][:3]
                gpu_lcs[k] = HBLikelihood(t, f, s, device=device)
            return gpu_lcs[k].light_curve(p[None, :])[0]

    samplers = [SlotSampler(niter, W, log10_periods[k], 0, W, run=run, npast=npast, ladder=ladder,
                            nthreads=nthreads) for k in range(K)]
    writers = [None] * K
    walkers_all = np.full(K, W, dtype=np.int32)
    t_ll = 0.0
    n_evals = 0

    def ev(P, walkers):
        nonlocal t_ll, n_evals
        t0 = time.perf_counter()
        out = np.asarray(loglik_multi(np.ascontiguousarray(P), walkers), dtype=np.float64)
        t_ll += time.perf_counter() - t0
        n_evals += len(P)
        return out

    try:
        x0 = [S.get()[0] for S in samplers]
        lmap = ev(np.stack([x[0] for x in x0]), np.ones(K, dtype=np.int32))  # :342, chain 0 of every target
        logLmap = [float(v) for v in lmap]
        xmap = [x[0].copy() for x in x0]
        if out_root:
            for k in range(K):
                root = os.path.join(out_root, str(run_ids[k]))
                writers[k] = Writer(root, run_ids[k], run, W)
                writers[k].attach(samplers[k])
        t_start = time.perf_counter()
        for it in range(int(niter)):
            Y = np.concatenate([S.propose(it) for S in samplers])
            if it == 0:
                lx = ev(np.concatenate([S.get()[0] for S in samplers]), walkers_all)
                for k, S in enumerate(samplers):
                    S.set_logl(lx[k * W:(k + 1) * W])
            ly = ev(Y, walkers_all)
            for k, S in enumerate(samplers):
                S.accept(it, ly[k * W:(k + 1) * W])
                _, Lcur, _ = S.get()
                perm, Lp = S.swap(Lcur)
                S.apply_perm(perm, None)
                if Lp[0] > logLmap[k]:  # :565-572
                    xmap[k] = S.get()[0][0].copy()
                    logLmap[k] = float(Lp[0])
                if it % 100 == 0 and writers[k] is not None:  # :593-649
                    xs = S.get()[0]
                    writers[k].step(it, Lp, xs)
                    t, f = targets[k][0], targets[k][1]
                    writers[k].light_curve(t, f, model(k, xmap[k]))
                    writers[k].pars(False, xs[0])
                S.end_iter(it)
            if verbose and it % 1000 == 0:
                print("%d/%d logLmap per target: %s" % (it, niter, " ".join("%.6g" % v for v in logLmap)))
        out = []
        for k, S in enumerate(samplers):
            if writers[k] is not None:  # :655-681
                t, f = targets[k][0], targets[k][1]
                writers[k].light_curve(t, f, model(k, xmap[k]))
                writers[k].pars(True, S.get()[0][0])
            st = S.stats()
            out.append({"run_id": run_ids[k], "xmap": xmap[k], "logLmap": logLmap[k], "accepted": st["cold_acc"],
                        "swaps": st["nswap"]})
        elapsed = time.perf_counter() - t_start
        for r in out:
            r.update(seconds_total=elapsed, seconds_loglik=t_ll, loglik_evals=n_evals)
        return out
    finally:
        for wtr in writers:
            if wtr is not None:
                wtr.close()
        for S in samplers:
            S.close()
        if gpu_cat is not None:
            gpu_cat.close()
        for L in gpu_lcs.values():
            L.close()


def deal_targets(ncad, world):
    """Targets -> ranks, largest first onto the least-loaded rank (cadence count)."""
    load = [0] * world
    owner = [0] * len(ncad)
    for k in sorted(range(len(ncad)), key=lambda i: -int(ncad[i])):
        r = min(range(world), key=lambda q: load[q])
        owner[k] = r
        load[r] += int(ncad[k])
    return owner


def main(argv=None):
    """python -m torch.distributed.run --nproc-per-node G -m hb_mcmc_amd.catalog NITER --root DIR
           --periods FILE [--targets TIC ...] [--chains W] ...
    FILE: lines "TIC log10P"; targets default to every TIC in FILE.  Inputs and
    outputs follow the reference tree (per target under DIR/<TIC>/)."""
    import argparse

    from .hbio import read_folded_lc, read_mag_file, read_periods

    ap = argparse.ArgumentParser(prog="hb_mcmc_amd.catalog")
    ap.add_argument("niter", type=int)
    ap.add_argument("--root", default=os.environ.get("HB_MCMC_ROOT", "."))
    ap.add_argument("--periods", required=True)
    ap.add_argument("--targets", nargs="*")
    ap.add_argument("--run", type=int, default=0)
    ap.add_argument("--chains", type=int, default=50)
    ap.add_argument("--npast", type=int, default=500)
    ap.add_argument("--ladder", type=int, default=0)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    periods = read_periods(a.periods)
    tics = a.targets or list(periods)
    data = []
    for tic in tics:
        lc = os.path.join(a.root, "data", "lightcurves", "folded_lightcurves", f"{tic}_new.txt")
        t, f, e = read_folded_lc(lc)
        mag, err = read_mag_file(os.path.join(a.root, "data", "magnitudes", f"{tic}.txt"))
        data.append((tic, (t, f, e, mag, err)))
    owner = deal_targets([len(d[1][0]) for d in data], world)
    mine = [d for d, o in zip(data, owner) if o == rank]
    if not mine:
        return 0
    import torch
    dev = local % max(1, torch.cuda.device_count())
    res = run_catalog([d[1] for d in mine], a.niter, [d[0] for d in mine], [periods[d[0]] for d in mine],
                      run=a.run, nchains=a.chains, npast=a.npast, ladder=a.ladder, nthreads=a.threads,
                      out_root=a.root, device=dev, verbose=not a.quiet)
    if not a.quiet:
        for r in res:
            print("rank %d target %s: logLmap %.12g, %d logL evals in %.3f s (%.3f s in the likelihood)" % (
                rank, r["run_id"], r["logLmap"], r["loglik_evals"], r["seconds_total"], r["seconds_loglik"]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
