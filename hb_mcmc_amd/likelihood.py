"""Batched heartbeat-binary log-likelihood on the GPU (Python mirror of the
hb_ctx C-ABI, include/hbmi.h Part 2).

``HBLikelihood(t, flux, sigma, mag_data, magerr)`` keeps one observed light
curve resident in HBM; ``loglike(params)`` evaluates W walkers (W x 21,
likelihood3.c:533-578 slot order) with the semantics of the reference
``loglikelihood`` (likelihood3.c:809-873) and ``light_curve(params)`` returns
the W x N model light curves of ``calc_light_curve`` (:530-686).

Inputs may be numpy arrays (host round trip, synchronous) or device-resident
torch tensors (``loglike_dev``/``light_curve_dev``: asynchronous on the
current torch stream, no host transfer).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .synth import MAG_DEFAULT, MAGERR_DEFAULT

NPARS = 21


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class HBLikelihood:
    def __init__(self, t, flux, sigma, mag_data=None, magerr=None, device: int = 0, latency_plan: bool = False):
        self.lib = _lib.lib()
        t, flux, sigma = _f64(t), _f64(flux), _f64(sigma)
        if not (t.shape == flux.shape == sigma.shape) or t.ndim != 1:
            raise ValueError("t, flux, sigma must be 1-D arrays of equal length")
        mag = _f64(MAG_DEFAULT if mag_data is None else mag_data)
        err = _f64(MAGERR_DEFAULT if magerr is None else magerr)
        if mag.shape != (5,) or err.shape != (4,):
            raise ValueError("mag_data must have 5 entries and magerr 4")
        self.n = int(t.shape[0])
        self.device = device
        pd = C.POINTER(C.c_double)
        h = self.lib.hb_create(t.ctypes.data_as(pd), flux.ctypes.data_as(pd), sigma.ctypes.data_as(pd),
                               self.n, mag.ctypes.data_as(pd), err.ctypes.data_as(pd), device)
        if not h:
            raise _lib.HBMIError("hb_create: " + _lib.last_error())
        self._h = C.c_void_p(h)
        if latency_plan:  # multi-wave kernel for batches < 512 walkers (hb_ctx_set_latency_plan)
            self.lib.hb_ctx_set_latency_plan(self._h, 1)

    # -- bookkeeping --
    def close(self):
        if getattr(self, "_h", None):
            self.lib.hb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def waves_per_walker(self) -> int:
        return self.lib.hb_ctx_waves_per_walker(self._h)

    @property
    def template_in_lds(self) -> bool:
        return bool(self.lib.hb_ctx_template_in_lds(self._h))

    @property
    def eval_kernel(self) -> str:
        """Name of the eval kernel this light curve's plan launches."""
        kind = self.lib.hb_ctx_eval_kind(self._h)
        return ("hb_eval_wave_kernel", "hb_eval_block_kernel", "hb_eval_kernel")[kind]

    def fused_wpb(self, w: int) -> int:
        """Walkers per workgroup of the single fused launch loglike_dev makes
        for w walkers (records in the eval kernel's prologue), 0 when it makes
        two launches (prepare_dev + evaluate_dev)."""
        return int(self.lib.hb_ctx_fused_wpb(self._h, int(w)))

    def reserve(self, max_walkers: int):
        _lib.check(self.lib.hb_reserve(self._h, int(max_walkers)), "hb_reserve")

    # -- host arrays --
    def loglike(self, params) -> np.ndarray:
        P = _f64(params).reshape(-1, NPARS)
        out = np.empty(P.shape[0])
        _lib.check(self.lib.hb_loglik_batch(self._h, _p(P), P.shape[0], _p(out), None), "hb_loglik_batch")
        return out

    def light_curve(self, params) -> np.ndarray:
        P = _f64(params).reshape(-1, NPARS)
        out = np.empty((P.shape[0], self.n))
        _lib.check(self.lib.hb_light_curve_batch(self._h, _p(P), P.shape[0], _p(out), None),
                   "hb_light_curve_batch")
        return out

    # -- device tensors (torch, float64, contiguous, on this context's GPU) --
    @staticmethod
    def _stream_handle(stream):
        if stream is None:
            import torch
            stream = torch.cuda.current_stream()
        return C.c_void_p(stream.cuda_stream)

    def loglike_dev(self, params_dev, out_dev, stream=None):
        self._check_dev(params_dev, out_dev, out_dev.numel())
        _lib.check(self.lib.hb_loglik_batch_dev(self._h, C.c_void_p(params_dev.data_ptr()), params_dev.shape[0],
                                                C.c_void_p(out_dev.data_ptr()), self._stream_handle(stream)),
                   "hb_loglik_batch_dev")

    def prepare_dev(self, params_dev, stream=None):
        """First launch of loglike_dev (per-walker constants), for timing."""
        self._check_dev(params_dev, params_dev[:, 0], params_dev.shape[0])
        _lib.check(self.lib.hb_prepare_dev(self._h, C.c_void_p(params_dev.data_ptr()), params_dev.shape[0],
                                           self._stream_handle(stream)), "hb_prepare_dev")

    def evaluate_dev(self, w, out_dev, mode=0, stream=None):
        """Second launch of loglike_dev (model + median + chi^2), for timing."""
        _lib.check(self.lib.hb_evaluate_dev(self._h, int(w), C.c_void_p(out_dev.data_ptr()), int(mode),
                                            self._stream_handle(stream)), "hb_evaluate_dev")

    def light_curve_dev(self, params_dev, out_dev, stream=None):
        self._check_dev(params_dev, out_dev, out_dev.shape[0])
        if out_dev.dim() != 2 or out_dev.shape[1] != self.n:
            raise ValueError("out_dev must be W x N")
        _lib.check(self.lib.hb_light_curve_batch_dev(self._h, C.c_void_p(params_dev.data_ptr()),
                                                     params_dev.shape[0], C.c_void_p(out_dev.data_ptr()),
                                                     self._stream_handle(stream)),
                   "hb_light_curve_batch_dev")

    @staticmethod
    def _check_dev(params_dev, out_dev, wout):
        import torch
        for x in (params_dev, out_dev):
            if not (x.is_cuda and x.dtype == torch.float64 and (x.is_contiguous() or x.dim() == 1)):
                raise ValueError("device buffers must be contiguous float64 GPU tensors")
        if params_dev.dim() != 2 or params_dev.shape[1] != NPARS:
            raise ValueError("params must be W x 21")
        if wout != params_dev.shape[0]:
            raise ValueError("output length must equal the walker count")
