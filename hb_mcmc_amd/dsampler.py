"""Device-resident PT-MCMC (include/hb_sampler.h, hb_dsampler_*): the
mcmc_wrapper2.c iteration with proposals, walls, priors, likelihood, Hastings
test, history and tempering swaps all on the GPU, bit-identical to the host
loop (SlotSampler) it starts from and hands back to.

    S = SlotSampler(niter, W, log10P, 0, W, ...)
    with DeviceSampler(S, HBLikelihood(t, f, sigma)) as D:
        D.init_logl()
        for it in range(niter):
            D.step(it)          # enqueued, no host wait
        x, logl, xmap, logLmap, stats = D.gather()
        D.download()            # S now holds the device state

`run_mcmc_device(...)` is hb_mcmc_run_device: the whole reference loop with
its output files, the host joining only every 100 iterations.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .sampler import MCMCConfig, MCMCResult, SlotSampler, _declare, _ok, _pd


class DeviceSampler:
    def __init__(self, sampler: SlotSampler, likelihood):
        self.lib = _declare(_lib.lib())
        if sampler.lo != 0 or sampler.hi != sampler.W:
            raise ValueError("the device sampler needs a SlotSampler that owns every slot")
        self.S, self.L = sampler, likelihood
        self._h = self.lib.hb_dsampler_create(sampler._h, likelihood._h)
        if not self._h:
            raise _lib.HBMIError("hb_dsampler_create: " + _lib.last_error())

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hb_dsampler_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            raise _lib.HBMIError(f"{what} failed ({rc}): {_lib.last_error()}")

    def init_logl(self):
        self._check(self.lib.hb_dsampler_init_logl(self._h), "hb_dsampler_init_logl")

    def step(self, it):
        self._check(self.lib.hb_dsampler_step(self._h, int(it)), "hb_dsampler_step")

    def sync(self):
        self._check(self.lib.hb_dsampler_sync(self._h), "hb_dsampler_sync")

    def gather(self):
        W = self.S.W
        x, ll, xmap = np.empty((W, 21)), np.empty(W), np.empty(21)
        lmap = C.c_double()
        st = (C.c_long * 4)()
        self._check(self.lib.hb_dsampler_gather(self._h, _pd(x), _pd(ll), _pd(xmap), C.byref(lmap), st),
                    "hb_dsampler_gather")
        return x, ll, xmap, lmap.value, dict(zip(("acc", "DEacc", "DEtrial", "atrial"), st[:]))

    def download(self):
        self._check(self.lib.hb_dsampler_download(self._h), "hb_dsampler_download")

    def host_times(self):
        """Host seconds since creation: schedule building (all producer
        threads), waits for a schedule, kernel issue; and the thread count."""
        out = np.zeros(4)
        self._check(self.lib.hb_dsampler_host_times(self._h, _pd(out)), "hb_dsampler_host_times")
        return {"sched_build": out[0], "sched_wait": out[1], "issue": out[2], "threads": int(out[3])}


def run_mcmc_device(t, flux, sigma, niter, run_id, log10_period, run=0, nchains=50, npast=500, ladder=0,
                    verbose=False, out_root=None, mag_data=None, magerr=None, device=0):
    """hb_mcmc_run_device (the reference loop, device-resident) over one light curve."""
    from .likelihood import HBLikelihood

    lib = _declare(_lib.lib())
    t = np.ascontiguousarray(t, dtype=np.float64)
    flux = np.ascontiguousarray(flux, dtype=np.float64)
    cfg = MCMCConfig(int(niter), int(nchains), int(npast), int(run), float(log10_period), int(ladder), 0,
                     int(bool(verbose)), (out_root or "").encode(), str(run_id).encode())
    res = MCMCResult()
    with HBLikelihood(t, flux, sigma, mag_data, magerr, device=device) as L:
        rc = lib.hb_mcmc_run_device(C.byref(cfg), L._h, _pd(t), _pd(flux), len(t), C.byref(res))
        _ok(rc, "hb_mcmc_run_device")
    return {"xmap": np.array(res.xmap[:]), "logLmap": res.logLmap, "accepted": res.accepted, "swaps": res.swaps,
            "seconds_total": res.seconds_total, "loglik_evals": res.loglik_evals}


class ShardedDeviceSampler:
    """One rank's share of the device-resident PT-MCMC (hb_dsampler_create_shard):
    this rank's GPU proposes, evaluates and tests the slots [W r/R, W (r+1)/R)
    of the ladder; per iteration ONE all-gather carries every rank's logL by
    slot and the records of the chains near its shard's edges, then every rank
    replays the tempering swaps inside its cone [lo - nlv, hi + nlv) (nlv = the
    iteration's dependency levels: no chain moves farther) on the cone's
    slice of index[] (mcmc_wrapper2.c:554-563).  The collective runs device to device on the
    sampler's own HIP stream under RCCL (backend "nccl"); under gloo (ranks
    sharing a GPU, rehearsal) it is staged through host memory.

        S = SlotSampler(niter, W, log10P, lo, hi, ...)      # lo, hi = dist.shard(W, rank, R)
        with ShardedDeviceSampler(S, HBLikelihood(...)) as D:
            D.init_logl()
            for it in range(niter):
                D.step(it)                                   # no host wait under RCCL
            x, logl, xmap, logLmap, stats = D.gather()       # this rank's slots

    exchange: run step_begin -> all-gather -> step_end even on one rank
    (default: only when R > 1; a one-rank sampler otherwise takes the plain
    hb_dsampler_step).  With backend "nccl" and R = 1 that is a real RCCL
    all-gather of world size 1 on the sampler's stream -- the ordering of
    ds_pack -> RCCL -> ds_swap that C4 relies on, testable on one GPU.
    """

    def __init__(self, sampler: SlotSampler, likelihood, group=None, exchange=None):
        import torch
        import torch.distributed as dist

        from .dist import shard

        self.lib = _declare(_lib.lib())
        self.torch, self.dist, self.group = torch, dist, group
        self.R, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.backend = dist.get_backend(group)
        W = sampler.W
        if (sampler.lo, sampler.hi) != shard(W, self.rank, self.R):
            raise ValueError(f"rank {self.rank} must own slots {shard(W, self.rank, self.R)}")
        self.S, self.L = sampler, likelihood
        counts = [hi - lo for lo, hi in (shard(W, q, self.R) for q in range(self.R))]
        self.counts = counts
        _, _, cid = sampler.get()
        chain_of_slot = np.ascontiguousarray(self._gather_rows(cid.astype(np.float64), counts).astype(np.int32))
        self.device = torch.device("cuda", likelihood.device)
        self.exchange = self.R > 1 if exchange is None else bool(exchange)
        if self.R > 1 and not self.exchange:
            raise ValueError("a sharded sampler always exchanges")
        if self.exchange:
            self._h = self.lib.hb_dsampler_create_shard(sampler._h, likelihood._h,
                                                        chain_of_slot.ctypes.data_as(C.POINTER(C.c_int)),
                                                        self.R, self.rank)
        else:
            self._h = self.lib.hb_dsampler_create(sampler._h, likelihood._h)
        if not self._h:
            raise _lib.HBMIError("hb_dsampler_create_shard: " + _lib.last_error())
        self.cap = int(self.lib.hb_dsampler_exchange_cap(self._h))
        self.send = torch.zeros(self.cap, dtype=torch.float64, device=self.device)
        self.recv = torch.zeros(self.R * self.cap, dtype=torch.float64, device=self.device)
        self.stream = torch.cuda.ExternalStream(self.lib.hb_dsampler_stream(self._h), device=self.device)
        self.exchanged_doubles = 0

    def _gather_rows(self, local, counts):
        """Small host-side all-gather of per-slot rows (setup, files)."""
        torch, dist = self.torch, self.dist
        m = max(counts)
        row = local.shape[1:]
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        buf = torch.zeros((m,) + tuple(row), dtype=torch.float64, device=dev)
        if len(local):
            buf[:len(local)] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64)).to(dev)
        out = torch.empty((self.R * m,) + tuple(row), dtype=torch.float64, device=dev)
        dist.all_gather_into_tensor(out, buf, group=self.group)
        out = out.cpu().numpy()
        return np.concatenate([out[r * m:r * m + c] for r, c in enumerate(counts)])

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hb_dsampler_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            raise _lib.HBMIError(f"{what} failed ({rc}): {_lib.last_error()}")

    def init_logl(self):
        self._check(self.lib.hb_dsampler_init_logl(self._h), "hb_dsampler_init_logl")

    def step(self, it):
        if not self.exchange:
            self._check(self.lib.hb_dsampler_step(self._h, int(it)), "hb_dsampler_step")
            return
        n = int(self.lib.hb_dsampler_step_begin(self._h, int(it), C.c_void_p(self.send.data_ptr()), self.cap))
        if n <= 0:
            raise _lib.HBMIError(f"hb_dsampler_step_begin failed ({n}): {_lib.last_error()}")
        R = self.R
        if self.backend == "nccl":
            # RCCL on the sampler's stream: ordered after ds_pack, and ds_swap after the gather
            with self.torch.cuda.stream(self.stream):
                self.dist.all_gather_into_tensor(self.recv[:R * n], self.send[:n], group=self.group)
        else:
            self._check(self.lib.hb_dsampler_sync(self._h), "hb_dsampler_sync")
            out = self.torch.empty(R * n, dtype=self.torch.float64)
            self.dist.all_gather_into_tensor(out, self.send[:n].cpu(), group=self.group)
            with self.torch.cuda.stream(self.stream):
                self.recv[:R * n].copy_(out)
        self.exchanged_doubles += n
        self._check(self.lib.hb_dsampler_step_end(self._h, int(it), C.c_void_p(self.recv.data_ptr()), n),
                    "hb_dsampler_step_end")

    def sync(self):
        self._check(self.lib.hb_dsampler_sync(self._h), "hb_dsampler_sync")

    def gather(self):
        """States / logL of this rank's slots, the MAP tracker (meaningful on
        the rank owning slot 0) and this rank's {acc, DEacc, DEtrial, atrial}."""
        nl = self.S.nl
        x, ll, xmap = np.empty((nl, 21)), np.empty(nl), np.empty(21)
        lmap = C.c_double()
        st = (C.c_long * 4)()
        self._check(self.lib.hb_dsampler_gather(self._h, _pd(x), _pd(ll), _pd(xmap), C.byref(lmap), st),
                    "hb_dsampler_gather")
        return x, ll, xmap, lmap.value, dict(zip(("acc", "DEacc", "DEtrial", "atrial"), st[:]))

    def gather_all(self):
        """(x, logL) of every slot, all-gathered to every rank."""
        x, ll, xmap, lmap, st = self.gather()
        return self._gather_rows(x, self.counts), self._gather_rows(ll, self.counts), xmap, lmap, st

    def download(self):
        self._check(self.lib.hb_dsampler_download(self._h), "hb_dsampler_download")

    def host_times(self):
        """Host seconds since creation: schedule building (all producer
        threads), waits for a schedule, kernel issue; and the thread count."""
        out = np.zeros(4)
        self._check(self.lib.hb_dsampler_host_times(self._h, _pd(out)), "hb_dsampler_host_times")
        return {"sched_build": out[0], "sched_wait": out[1], "issue": out[2], "threads": int(out[3])}
