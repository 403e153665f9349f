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
