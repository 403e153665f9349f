"""Python front end of the PT-MCMC caller (include/hb_sampler.h), i.e. the
sidruns30/HB_MCMC sampler loop of src/mcmc_wrapper2.c with one batched
likelihood call per step.

    res = run_mcmc(t, flux, sigma, niter=1200, run_id="127079833",
                   log10_period=0.5021, out_root="/path/root")

By default the likelihood and the .out model curve come from the GPU
(HBLikelihood on libhbmi.so).  `loglik(P) -> logL[W]` and `model(p) -> m[n]`
may be supplied instead (any provider with the reference's semantics).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

LOGLIK_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double))
MODEL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double))


class MCMCConfig(C.Structure):
    _fields_ = [("niter", C.c_long), ("nchains", C.c_int), ("npast", C.c_int), ("run", C.c_int),
                ("log10_period", C.c_double), ("ladder", C.c_int), ("nthreads", C.c_int), ("verbose", C.c_int),
                ("out_root", C.c_char_p), ("run_id", C.c_char_p)]


class MCMCResult(C.Structure):
    _fields_ = [("xmap", C.c_double * 21), ("logLmap", C.c_double), ("accepted", C.c_long), ("swaps", C.c_long),
                ("seconds_total", C.c_double), ("seconds_loglik", C.c_double), ("loglik_evals", C.c_long)]


def _declare(lib):
    if getattr(lib, "_hb_sampler_declared", False):
        return lib
    lib.hb_mcmc_run.restype = C.c_int
    lib.hb_mcmc_run.argtypes = [C.POINTER(MCMCConfig), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                C.POINTER(C.c_double), C.c_long, LOGLIK_FN, MODEL_FN, C.c_void_p,
                                C.POINTER(MCMCResult)]
    lib.hb_ran2_parallel.restype = C.c_double
    lib.hb_ran2_parallel.argtypes = [C.POINTER(C.c_long), C.c_void_p]
    lib.hb_gasdev2_parallel.restype = C.c_double
    lib.hb_gasdev2_parallel.argtypes = [C.POINTER(C.c_long), C.c_void_p]
    lib.hb_rand_stream.restype = C.c_int
    lib.hb_rand_stream.argtypes = [C.c_uint, C.c_int, C.POINTER(C.c_int)]
    vp, pd, pi = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)
    for name, res, args in (
            ("hb_sampler_create", vp, [C.POINTER(MCMCConfig), C.c_int, C.c_int]),
            ("hb_sampler_destroy", None, [vp]),
            ("hb_sampler_attach_log", C.c_int, [vp, vp]),
            ("hb_sampler_get", C.c_int, [vp, pd, pd, pi]),
            ("hb_sampler_set_logl", C.c_int, [vp, pd]),
            ("hb_sampler_propose", C.c_int, [vp, C.c_long, pd]),
            ("hb_sampler_accept", C.c_int, [vp, C.c_long, pd]),
            ("hb_sampler_swap", C.c_int, [vp, pd, pi, pd]),
            ("hb_sampler_pack", C.c_int, [vp, C.c_int, pd]),
            ("hb_sampler_apply_perm", C.c_int, [vp, pi, pd]),
            ("hb_sampler_stats", C.c_int, [vp, C.POINTER(C.c_long)]),
            ("hb_sampler_end_iter", C.c_int, [vp, C.c_long]),
            ("hb_sampler_export", C.c_int, [vp, C.POINTER(C.c_long), vp, pd]),
            ("hb_dsampler_create", vp, [vp, vp]),
            ("hb_dsampler_destroy", None, [vp]),
            ("hb_dsampler_init_logl", C.c_int, [vp]),
            ("hb_dsampler_step", C.c_int, [vp, C.c_long]),
            ("hb_dsampler_gather", C.c_int, [vp, pd, pd, pd, pd, C.POINTER(C.c_long)]),
            ("hb_dsampler_sync", C.c_int, [vp]),
            ("hb_dsampler_download", C.c_int, [vp]),
            ("hb_dsampler_create_shard", vp, [vp, vp, pi, C.c_int, C.c_int]),
            ("hb_dsampler_step_begin", C.c_long, [vp, C.c_long, vp, C.c_long]),
            ("hb_dsampler_step_end", C.c_int, [vp, C.c_long, vp, C.c_long]),
            ("hb_dsampler_exchange_cap", C.c_long, [vp]),
            ("hb_dsampler_stream", vp, [vp]),
            ("hb_dsampler_host_times", C.c_int, [vp, pd]),
            ("hb_rand_stream_jump", C.c_int, [C.c_uint, C.c_ulonglong, C.c_int, C.POINTER(C.c_int)]),
            ("hb_mcmc_run_device", C.c_int, [C.POINTER(MCMCConfig), vp, pd, pd, C.c_long, C.POINTER(MCMCResult)]),
            ("hb_glibc_eval", C.c_int, [C.c_int, pd, pd, C.c_long, pd]),
            ("hb_writer_open", vp, [C.c_char_p, C.c_char_p, C.c_int, C.c_int]),
            ("hb_writer_step", C.c_int, [vp, C.c_long, pd, pd]),
            ("hb_writer_lc", C.c_int, [vp, pd, pd, pd, C.c_long]),
            ("hb_writer_pars", C.c_int, [vp, C.c_int, pd]),
            ("hb_writer_close", None, [vp])):
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    lib._hb_sampler_declared = True
    return lib


REC = 23  # HB_SAMPLER_REC: x[21], logL, chain id
RNG_VARS_BYTES = 8 * 34 + 8 + 8 + 8  # struct RNG_Vars: idum2, iy, iv[32], iset (+pad), gset, cts


def _pd(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ok(rc, what):
    if rc != 0:
        raise _lib.HBMIError(f"{what} failed ({rc})")


class SlotSampler:
    """The phase API of include/hb_sampler.h for temperature slots [lo, hi)
    of an `nchains` ladder (one rank's share; lo=0, hi=nchains = everything)."""

    def __init__(self, niter, nchains, log10_period, lo, hi, run=0, npast=500, ladder=0, nthreads=0):
        self.lib = _declare(_lib.lib())
        self.cfg = MCMCConfig(int(niter), int(nchains), int(npast), int(run), float(log10_period), int(ladder),
                              int(nthreads), 0, b"", b"run")
        self.W, self.lo, self.hi, self.nl = int(nchains), int(lo), int(hi), int(hi) - int(lo)
        self._h = self.lib.hb_sampler_create(C.byref(self.cfg), self.lo, self.hi)
        if not self._h:
            raise _lib.HBMIError("hb_sampler_create rejected the configuration")
        self.y = np.empty((self.nl, 21))
        self.perm = np.empty(self.W, dtype=np.int32)
        self.logl_perm = np.empty(self.W)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hb_sampler_destroy(self._h)
            self._h = None

    __del__ = close

    def get(self):
        x, ll, cid = np.empty((self.nl, 21)), np.empty(self.nl), np.empty(self.nl, dtype=np.int32)
        _ok(self.lib.hb_sampler_get(self._h, _pd(x), _pd(ll), cid.ctypes.data_as(C.POINTER(C.c_int))),
            "hb_sampler_get")
        return x, ll, cid

    def set_logl(self, logl):
        logl = np.ascontiguousarray(logl, dtype=np.float64)
        _ok(self.lib.hb_sampler_set_logl(self._h, _pd(logl)), "hb_sampler_set_logl")

    def propose(self, it):
        _ok(self.lib.hb_sampler_propose(self._h, int(it), _pd(self.y)), "hb_sampler_propose")
        return self.y

    def accept(self, it, logly):
        logly = np.ascontiguousarray(logly, dtype=np.float64)
        _ok(self.lib.hb_sampler_accept(self._h, int(it), _pd(logly)), "hb_sampler_accept")

    def swap(self, logl_all):
        logl_all = np.ascontiguousarray(logl_all, dtype=np.float64)
        n = self.lib.hb_sampler_swap(self._h, _pd(logl_all), self.perm.ctypes.data_as(C.POINTER(C.c_int)),
                                     _pd(self.logl_perm))
        if n < 0:
            raise _lib.HBMIError("hb_sampler_swap failed")
        return self.perm, self.logl_perm

    def pack(self, slots):
        out = np.empty((len(slots), REC))
        for i, j in enumerate(slots):
            _ok(self.lib.hb_sampler_pack(self._h, int(j), _pd(out[i])), "hb_sampler_pack")
        return out

    def apply_perm(self, perm, remote=None):
        perm = np.ascontiguousarray(perm, dtype=np.int32)
        rp = None if remote is None else _pd(np.ascontiguousarray(remote, dtype=np.float64))
        _ok(self.lib.hb_sampler_apply_perm(self._h, perm.ctypes.data_as(C.POINTER(C.c_int)), rp),
            "hb_sampler_apply_perm")

    def stats(self):
        out = (C.c_long * 6)()
        _ok(self.lib.hb_sampler_stats(self._h, out), "hb_sampler_stats")
        return dict(zip(("acc", "DEacc", "DEtrial", "atrial", "cold_acc", "nswap"), out[:]))

    def end_iter(self, it):
        _ok(self.lib.hb_sampler_end_iter(self._h, int(it)), "hb_sampler_end_iter")

    def state_arrays(self):
        """RNG streams (seeds, raw RNG_Vars records) and history of the owned slots."""
        seeds = np.empty(self.nl, dtype=np.int64)
        states = np.empty((self.nl, RNG_VARS_BYTES), dtype=np.uint8)
        hist = np.empty((self.nl, self.cfg.npast, 21))
        _ok(self.lib.hb_sampler_export(self._h, seeds.ctypes.data_as(C.POINTER(C.c_long)),
                                       states.ctypes.data_as(C.c_void_p), _pd(hist)), "hb_sampler_export")
        return {"seeds": seeds, "rng_states": states, "history": hist}


class Writer:
    """The reference's output files (mcmc_wrapper2.c:110-173, :593-681)."""

    def __init__(self, root, run_id, run, nchains):
        self.lib = _declare(_lib.lib())
        self._h = self.lib.hb_writer_open(str(root).encode(), str(run_id).encode(), int(run), int(nchains))
        if not self._h:
            raise _lib.HBMIError(f"cannot open the output tree under {root}")

    def attach(self, sampler: SlotSampler):
        _ok(self.lib.hb_sampler_attach_log(sampler._h, self._h), "hb_sampler_attach_log")

    def step(self, it, logl_slots, x_slots):
        a = np.ascontiguousarray(logl_slots, dtype=np.float64)
        b = np.ascontiguousarray(x_slots, dtype=np.float64)
        _ok(self.lib.hb_writer_step(self._h, int(it), _pd(a), _pd(b)), "hb_writer_step")

    def light_curve(self, t, f, m):
        t, f, m = (np.ascontiguousarray(v, dtype=np.float64) for v in (t, f, m))
        _ok(self.lib.hb_writer_lc(self._h, _pd(t), _pd(f), _pd(m), len(t)), "hb_writer_lc")

    def pars(self, final, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        _ok(self.lib.hb_writer_pars(self._h, int(bool(final)), _pd(x)), "hb_writer_pars")

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hb_writer_close(self._h)
            self._h = None


def run_mcmc(t, flux, sigma, niter, run_id, log10_period, run=0, nchains=50, npast=500, ladder=0, nthreads=0,
             verbose=False, out_root=None, loglik=None, model=None, mag_data=None, magerr=None, device=0):
    lib = _declare(_lib.lib())
    t = np.ascontiguousarray(t, dtype=np.float64)
    flux = np.ascontiguousarray(flux, dtype=np.float64)
    sigma = np.ascontiguousarray(sigma, dtype=np.float64)
    n = len(t)
    gpu = None
    if loglik is None or model is None:
        from .likelihood import HBLikelihood

        gpu = HBLikelihood(t, flux, sigma, mag_data, magerr, device=device)
        gpu.reserve(nchains)
        loglik = loglik or gpu.loglike
        model = model or (lambda p: gpu.light_curve(p[None, :])[0])
    err = []

    def _ll(_, P, w, out):
        try:
            arr = np.ctypeslib.as_array(P, shape=(w * 21,)).reshape(w, 21).copy()
            res = np.asarray(loglik(arr), dtype=np.float64)
            np.ctypeslib.as_array(out, shape=(w,))[:] = res
            return 0
        except Exception as e:  # noqa: BLE001 -- surfaced after the run
            err.append(e)
            return 1

    def _model(_, p, out):
        try:
            arr = np.ctypeslib.as_array(p, shape=(21,)).copy()
            np.ctypeslib.as_array(out, shape=(n,))[:] = np.asarray(model(arr), dtype=np.float64)
            return 0
        except Exception as e:  # noqa: BLE001
            err.append(e)
            return 1

    cfg = MCMCConfig(int(niter), int(nchains), int(npast), int(run), float(log10_period), int(ladder), int(nthreads),
                     int(bool(verbose)), (out_root or "").encode(), str(run_id).encode())
    res = MCMCResult()
    ll_cb, m_cb = LOGLIK_FN(_ll), MODEL_FN(_model)
    pd = C.POINTER(C.c_double)
    rc = lib.hb_mcmc_run(C.byref(cfg), t.ctypes.data_as(pd), flux.ctypes.data_as(pd), sigma.ctypes.data_as(pd), n,
                         ll_cb, m_cb, None, C.byref(res))
    if gpu is not None:
        gpu.close()
    if err:
        raise err[0]
    if rc != 0:
        raise _lib.HBMIError(f"hb_mcmc_run failed ({rc})")
    return {"xmap": np.array(res.xmap[:]), "logLmap": res.logLmap, "accepted": res.accepted, "swaps": res.swaps,
            "seconds_total": res.seconds_total, "seconds_loglik": res.seconds_loglik,
            "loglik_evals": res.loglik_evals}
