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
    lib._hb_sampler_declared = True
    return lib


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
