"""glibc-exact exp/log/pow (hb_mcmc_amd/csrc/hb_glibc_math.hpp) against the
system libm, bit for bit.

The device sampler draws the reference's proposals through these functions
(jump scale pow(10, .) mcmc_wrapper2.c:391, polar Gaussian log :966, priors
:761/:1175-1178, Hastings exp :492, tempering exp :810), so they must equal
glibc's results on every argument the sampler can produce.  CPU: the host
build of the same header against libm on a few million arguments per
function, covering every branch (near 1, subnormal, under/overflow, negative
bases, integer exponents).  GPU: the device build against libm.
"""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hb_mcmc_amd", "lib", "libhbglibc_check.so")
pd = C.POINTER(C.c_double)


def _lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run __graft_entry__.build()")
    lib = C.CDLL(LIB)
    lib.hbg_check.restype = C.c_long
    lib.hbg_check.argtypes = [C.c_int, pd, pd, C.c_long, C.POINTER(C.c_long)]
    lib.hbg_libm.argtypes = [C.c_int, pd, pd, C.c_long, pd]
    return lib


def _args(fn, n, seed):
    """Arguments exercising every branch of fn (0 exp, 1 log, 2 pow)."""
    rng = np.random.default_rng(seed)
    if fn == 0:
        x = np.concatenate([
            rng.uniform(-750, 720, n // 4),                  # whole finite range incl. subnormal results
            rng.uniform(-746, -700, n // 8),                 # subnormal/underflow special case
            rng.uniform(700, 710, n // 16),                  # overflow special case
            rng.normal(0, 1, n // 4),                         # Hastings / tempering arguments
            -0.5 * rng.normal(0, 30, n // 8) ** 2,            # Gaussian prior exponents
            np.ldexp(rng.uniform(-1, 1, n // 16), rng.integers(-80, -40, n // 16)),  # tiny
            [0.0, -0.0, np.inf, -np.inf, np.nan, 1e308, -1e308, 709.782712893384, -745.1332191019411],
        ])
        y = np.zeros_like(x)
    elif fn == 1:
        bits = rng.integers(1, 0x7FF0000000000000, n // 4, dtype=np.int64).view(np.float64)  # all positive doubles
        x = np.concatenate([
            bits,
            rng.uniform(0.9, 1.1, n // 4),                   # near-1 branch
            rng.uniform(0, 1, n // 4),                        # Marsaglia rsq
            np.exp(-rng.uniform(0, 700, n // 8)),             # prior densities
            np.ldexp(rng.uniform(1, 2, n // 16), rng.integers(-1074, -1022, n // 16)),  # subnormal
            [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 5e-324],
        ])
        y = np.zeros_like(x)
    else:
        m = n // 8
        x = np.concatenate([
            np.full(m, 10.0), rng.normal(0, 1e3, m), rng.normal(0, 1, m),
            np.abs(rng.normal(0, 10, m)), rng.integers(1, 0x7FF0000000000000, m, dtype=np.int64).view(np.float64),
            -np.abs(rng.normal(0, 10, m)), rng.normal(0, 1e-150, m), rng.normal(0, 1e160, m),
            [0.0, -0.0, -2.0, -2.0, 1.0, np.inf, np.nan, 10.0],
        ])
        y = np.concatenate([
            rng.uniform(-6, 0, m), np.full(m, 2.0), np.full(m, 2.0),
            rng.normal(0, 30, m), rng.uniform(-2, 2, m),
            rng.integers(-40, 40, m).astype(np.float64), np.full(m, 2.0), np.full(m, 2.0),
            [2.0, 3.0, 3.0, 0.5, np.nan, -1.0, 2.0, -400.0],
        ])
    return np.ascontiguousarray(x), np.ascontiguousarray(y)


@pytest.mark.parametrize("fn,name", [(0, "exp"), (1, "log"), (2, "pow")])
def test_port_equals_libm(fn, name):
    lib = _lib()
    for seed in range(4):
        x, y = _args(fn, 1 << 20, seed)
        first = C.c_long()
        bad = lib.hbg_check(fn, x.ctypes.data_as(pd), y.ctypes.data_as(pd), len(x), C.byref(first))
        if bad:
            i = first.value
            ref = np.empty(1)
            lib.hbg_libm(fn, x[i:i + 1].ctypes.data_as(pd), y[i:i + 1].ctypes.data_as(pd), 1, ref.ctypes.data_as(pd))
            pytest.fail(f"{name}: {bad} of {len(x)} differ from libm; first x={x[i]!r} y={y[i]!r} libm={ref[0]!r}")


@pytest.mark.gpu
@pytest.mark.parametrize("fn,name", [(0, "exp"), (1, "log"), (2, "pow"), (3, "sqrt"), (4, "div")])
def test_device_equals_libm(fn, name):
    from hb_mcmc_amd import _lib as L
    from hb_mcmc_amd import sampler

    lib = _lib()
    hb = sampler._declare(L.lib())
    x, y = _args(min(fn, 2), 1 << 20, 11)
    if fn == 3:
        x = np.abs(x)
    if fn == 4:
        y = np.where(y == 0, 3.0, y)
    got = np.empty_like(x)
    rc = hb.hb_glibc_eval(fn, x.ctypes.data_as(pd), y.ctypes.data_as(pd), len(x), got.ctypes.data_as(pd))
    assert rc == 0
    ref = np.empty_like(x)
    if fn <= 2:
        lib.hbg_libm(fn, x.ctypes.data_as(pd), y.ctypes.data_as(pd), len(x), ref.ctypes.data_as(pd))
    elif fn == 3:
        ref = np.sqrt(x)
    else:
        ref = x / y
    same = (got.view(np.int64) == ref.view(np.int64)) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), f"{name}: {np.count_nonzero(~same)} differ; first x={x[~same][0]!r} y={y[~same][0]!r}"
