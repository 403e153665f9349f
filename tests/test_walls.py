"""Reflecting / periodic walls (mcmc_wrapper2.c:440-467): the exact
fast-forward of long reflection runs (hb_mcmc_amd/csrc/hb_walls.hpp, used by
the host and the device sampler) against the plain one-fold-at-a-time loop,
bit for bit -- the set_limits ranges (likelihood3.c:986-1120), random ranges,
grid-tie ranges, huge excursions and the 10^8-fold guard."""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hb_mcmc_amd", "lib", "libhbglibc_check.so")
pd = C.POINTER(C.c_double)

# set_limits (likelihood3.c:986-1120): (lo, hi) per slot
LIMITS = [(-1.5, 2.0), (-1.5, 2.0), (-2.0, 3.0), (0.0, 1.0), (0.0, np.pi), (-np.pi, np.pi), (0.0, 2.0691),
          (-5.0, 5.0), (-5.0, 5.0), (0.12, 0.20), (0.3, 0.38), (0.12, 0.20), (0.3, 0.38), (0.5, 1.5), (0.5, 1.5),
          (-0.3, 0.3), (-0.3, 0.3), (-5.0, 5.0), (-5.0, 5.0), (0.0, 1.0), (0.99, 1.01)]


def run(plain, v, lo, hi, fl, fh):
    lib = C.CDLL(LIB)
    lib.hbw_eval.argtypes = [C.c_int, pd, pd, pd, pd, pd, C.c_long, pd]
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (v, lo, hi, fl, fh)]
    out = np.empty(len(arrs[0]))
    lib.hbw_eval(plain, *[a.ctypes.data_as(pd) for a in arrs], len(out), out.ctypes.data_as(pd))
    return out


def check(v, lo, hi, fl, fh):
    a = run(0, v, lo, hi, fl, fh)
    b = run(1, v, lo, hi, fl, fh)
    same = (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    if not same.all():
        i = int(np.nonzero(~same)[0][0])
        pytest.fail(f"{np.count_nonzero(~same)} differ; v={v[i]!r} lo={lo[i]!r} hi={hi[i]!r} "
                    f"ff={a[i]!r} plain={b[i]!r}")
    return a


def test_set_limits_ranges_hot_chain_excursions():
    rng = np.random.default_rng(1)
    n = 20000
    k = rng.integers(0, len(LIMITS), n)
    lo = np.array([LIMITS[i][0] for i in k])
    hi = np.array([LIMITS[i][1] for i in k])
    width = hi - lo
    dist = width * 10 ** rng.uniform(-3, 4, n)          # up to 10^4 ranges: up to ~10^4 folds
    side = rng.integers(0, 2, n)
    v = np.where(side == 1, hi + dist, lo - dist)
    out = check(v, lo, hi, np.ones(n), np.ones(n))
    assert np.all((out >= lo) & (out <= hi))


def test_random_ranges_and_grid_ties():
    rng = np.random.default_rng(2)
    n = 20000
    lo = np.concatenate([rng.normal(0, 3, n // 2), np.ldexp(rng.integers(-8, 8, n // 2), rng.integers(-3, 3, n // 2))])
    width = np.concatenate([10 ** rng.uniform(-4, 1, n // 2), np.ldexp(1.0, rng.integers(-4, 3, n // 2))])
    hi = lo + width
    dist = width * 10 ** rng.uniform(-2, 4.5, n)
    v = np.where(rng.integers(0, 2, n) == 1, hi + dist, lo - dist)
    check(v, lo, hi, np.ones(n), np.ones(n))


def test_negative_ranges_and_binade_edges():
    """Ranges below zero, straddling zero, and excursions starting exactly at
    powers of two (the fast-forward's binade boundaries)."""
    rng = np.random.default_rng(4)
    n = 20000
    hi = rng.normal(0, 2, n)
    lo = hi - 10 ** rng.uniform(-3, 0.5, n)
    lim = np.maximum(np.abs(lo), np.abs(hi))
    edge = np.ldexp(1.0, np.ceil(np.log2(2 * lim)).astype(int) + rng.integers(0, 12, n))
    jitter = rng.choice([0.0, 1.0, -1.0], n) * np.ldexp(1.0, -rng.integers(1, 60, n)) * edge
    v = np.where(rng.integers(0, 2, n) == 1, edge + jitter, -(edge + jitter))
    check(v, lo, hi, np.ones(n), np.ones(n))


def test_one_sided_and_periodic_walls():
    rng = np.random.default_rng(3)
    n = 5000
    lo, hi = np.full(n, -np.pi), np.full(n, np.pi)
    v = rng.normal(0, 50, n)
    for fl, fh in ((1, 0), (0, 1), (2, 2), (1, 2), (2, 1), (0, 0)):
        check(v, lo, hi, np.full(n, fl), np.full(n, fh))


def test_fold_guard_and_endless_runs():
    """|v| so large that the plain loop stops at its 10^8-fold guard (also the
    case where both walls round to the same grid point and the folds cycle)."""
    v = np.array([-1.0e12, 3.0e11, 1.0e20, -7.5e17])
    lo = np.array([0.12, 0.3, 0.12, -1.5])
    hi = np.array([0.20, 0.38, 0.20, 2.0])
    check(v, lo, hi, np.ones(4), np.ones(4))


def test_tie_binades_within_reach():
    """Bounds whose doubled value is a half-integer number of ulps in a binade
    the excursion crosses (lo = odd * 2^(eb-54), eb in [1, 10]): the folds of
    those binades round half to even (hb_walls.hpp tie_double_folds)."""
    rng = np.random.default_rng(5)
    n = 20000
    eb = rng.integers(1, 11, n)
    span = np.ldexp(1.0, 54 - eb)
    odd = np.floor(rng.uniform(0.05, 2.0, n) * span / 2) * 2 + 1
    lo = np.ldexp(odd, eb - 54) * np.where(rng.integers(0, 2, n) == 1, 1.0, -1.0)
    width = 10 ** rng.uniform(-2, 0.5, n)
    hi = lo + width
    swap = rng.integers(0, 2, n) == 1  # the tie on the upper bound instead
    lo, hi = np.where(swap, lo - width, lo), np.where(swap, lo, hi)
    dist = width * 10 ** rng.uniform(1, 4, n)
    v = np.where(rng.integers(0, 2, n) == 1, hi + dist, lo - dist)
    out = check(v, lo, hi, np.ones(n), np.ones(n))
    assert np.all((out >= lo) & (out <= hi))


@pytest.mark.gpu
def test_device_walls_equal_plain_loop():
    """The device compile of hb_walls.hpp (hbx_wall_probe: ds_propose's
    apply_wall, one value per lane) against the host's plain loop, bit for bit,
    on the set_limits ranges with hot-chain excursions up to 10^5 ranges and
    on grid-tie ranges."""
    import sys
    sys.path.insert(0, ROOT)
    from hb_mcmc_amd import _lib

    lib = _lib.lib()
    f = lib.hbx_wall_probe
    f.argtypes = [pd, pd, pd, C.c_long, pd, C.POINTER(C.c_longlong)]
    f.restype = C.c_int
    rng = np.random.default_rng(7)
    n = 64 * 400
    k = rng.integers(0, len(LIMITS), n)
    lo = np.array([LIMITS[i][0] for i in k])
    hi = np.array([LIMITS[i][1] for i in k])
    # a quarter on grid-tie ranges (dyadic walls)
    t = rng.random(n) < 0.25
    lo[t] = np.ldexp(rng.integers(-8, 8, t.sum()), rng.integers(-3, 3, t.sum())).astype(float)
    hi[t] = lo[t] + np.ldexp(1.0, rng.integers(-4, 3, t.sum()))
    dist = (hi - lo) * 10 ** rng.uniform(-3, 5, n)
    v = np.where(rng.integers(0, 2, n) == 1, hi + dist, lo - dist)
    out = np.empty(n)
    cyc = np.empty((n + 63) // 64, dtype=np.int64)
    assert f(v.ctypes.data_as(pd), lo.ctypes.data_as(pd), hi.ctypes.data_as(pd), n, out.ctypes.data_as(pd),
             cyc.ctypes.data_as(C.POINTER(C.c_longlong))) == 0, _lib.last_error()
    ref = run(1, v, lo, hi, np.ones(n), np.ones(n))
    bad = out.view(np.int64) != ref.view(np.int64)
    assert not bad.any(), f"{bad.sum()} differ, first v={v[bad][0]!r} lo={lo[bad][0]!r} hi={hi[bad][0]!r}"
    assert np.all((out >= lo) & (out <= hi))
