"""Loader of libhbmi.so (the product's HIP library).

There is no CPU fallback: if the library is missing this raises, and if no
GPU is present the batched API reports an error from the HIP runtime.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HBMI_LIB") or os.path.join(PKG, "lib", "libhbmi.so")  # override: experiments only
CSRC = os.path.join(PKG, "csrc")

_D = C.c_double
_PD = C.POINTER(C.c_double)
_L = C.c_long
_I = C.c_int
_VP = C.c_void_p

_lock = threading.Lock()
_lib = None


class HBMIError(RuntimeError):
    pass


# sources that determine the likelihood kernels' machine code: the PMC counter
# file (profiles/pmc_counters.json) is keyed by this id, so bench.py only
# quotes counters that were measured on the kernels it runs
KERNEL_SOURCES = ("hb_kernels.hip", "hb_wave.hpp", "hb_device.hpp", "hb_math.hpp", "hb_internal.hpp",
                  "hb_accept.hpp", "hb_prep.hpp", "hb_glibc_math.hpp", "hb_glibc_tables.inc", "Makefile")


def kernel_build_id() -> str:
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(CSRC, name), "rb") as fh:
            h.update(name.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def build(jobs: int = 4) -> str:
    """Compile libhbmi.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", CSRC], check=True)
    return LIB_PATH


def _declare(lib):
    lib.hb_create.restype = _VP
    lib.hb_create.argtypes = [_PD, _PD, _PD, _L, _PD, _PD, _I]
    lib.hb_destroy.argtypes = [_VP]
    lib.hb_ctx_ncad.restype = _L
    lib.hb_ctx_ncad.argtypes = [_VP]
    lib.hb_reserve.restype = _I
    lib.hb_reserve.argtypes = [_VP, _I]
    for nm in ("hb_loglik_batch_dev", "hb_loglik_batch", "hb_light_curve_batch_dev", "hb_light_curve_batch"):
        f = getattr(lib, nm)
        f.restype = _I
        f.argtypes = [_VP, _VP, _I, _VP, _VP]
    lib.hb_prepare_dev.restype = _I
    lib.hb_prepare_dev.argtypes = [_VP, _VP, _I, _VP]
    lib.hb_evaluate_dev.restype = _I
    lib.hb_evaluate_dev.argtypes = [_VP, _I, _VP, _I, _VP]
    lib.hb_ctx_waves_per_walker.restype = _I
    lib.hb_ctx_waves_per_walker.argtypes = [_VP]
    lib.hb_ctx_template_in_lds.restype = _I
    lib.hb_ctx_template_in_lds.argtypes = [_VP]
    lib.hb_ctx_eval_kind.restype = _I
    lib.hb_ctx_eval_kind.argtypes = [_VP]
    lib.hb_ctx_fused_wpb.restype = _I
    lib.hb_ctx_fused_wpb.argtypes = [_VP, _I]
    lib.hb_ctx_set_latency_plan.restype = _I
    lib.hb_ctx_set_latency_plan.argtypes = [_VP, _I]
    lib.hb_last_error.restype = C.c_char_p
    lib.hb_device_available.restype = _I
    lib.hb_timer_create.restype = _VP
    lib.hb_timer_record.restype = _I
    lib.hb_timer_record.argtypes = [_VP, _VP]
    lib.hb_timer_elapsed_ms.restype = C.c_float
    lib.hb_timer_elapsed_ms.argtypes = [_VP, _VP]
    lib.hb_timer_destroy.argtypes = [_VP]
    # likelihood3.h drop-in symbols
    lib.loglikelihood.restype = _D
    lib.loglikelihood.argtypes = [_PD, _PD, _PD, _L, _PD, _PD, _PD]
    lib.calc_light_curve.argtypes = [_PD, _L, _PD, _PD]
    lib.traj.argtypes = [_PD, _PD, _PD, _PD, _PD, _PD, _PD, _I]
    for nm, n in (("get_alpha_beam", 1), ("beaming", 8), ("ellipsoidal", 11), ("reflection", 9),
                  ("eclipse_area", 3), ("_getT", 1), ("_getR", 1), ("envelope_Temp", 1),
                  ("envelope_Radius", 1), ("Eggleton_RL", 1)):
        f = getattr(lib, nm)
        f.restype = _D
        f.argtypes = [_D] * n
    lib.calc_radii_and_Teffs.argtypes = [_PD, _PD, _PD, _PD, _PD]
    lib.calc_mags.argtypes = [_PD, _D, _PD, _PD, _PD, _PD]
    lib.RocheOverflow.restype = _I
    lib.RocheOverflow.argtypes = [_PD]
    lib.remove_median.argtypes = [_PD, _L, _L]
    lib.quickSort.argtypes = [_PD, _I, _I]
    lib.partition.restype = _D
    lib.partition.argtypes = [_PD, _I, _I]
    lib.set_limits.argtypes = [_VP, _VP, _VP, _D]
    lib.initialize_proposals.argtypes = [_PD, _VP]
    # internal (tests, bench): drop-in bookkeeping (hb_dropin.hpp) and the
    # Kepler probe; absent from older builds loaded as A/B variants (HBMI_LIB)
    for name, res, args in (("hbx_dropin_stats", _I, [_PD, _I]), ("hbx_dropin_set_memo", _I, [_I]),
                            ("hbx_dropin_test_hash", _I, [_I]), ("hbx_kepler_probe", _I, [_PD, _L, _D, _I, _PD])):
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
    return lib


def lib():
    """The loaded libhbmi.so (raises HBMIError if it was never built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HBMIError(f"{LIB_PATH} not found: build it with `make -C {CSRC}` "
                                "(hb_mcmc_amd has no CPU fallback)")
            _lib = _declare(C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL))
        return _lib


def last_error() -> str:
    return lib().hb_last_error().decode(errors="replace")


def check(rc: int, what: str):
    if rc != 0:
        raise HBMIError(f"{what} failed ({rc}): {last_error()}")


def device_available() -> bool:
    return bool(lib().hb_device_available())
