"""The eclipse kernels' asin (hb_mcmc_amd/csrc/hb_device.hpp asin01, used by
overlap_partial for the reference's asin(hh / r), likelihood3.c:372-377):
its coefficients, read from the header, evaluated in the device's order
(numpy float64, mul + add standing in for each fma), stay within 3 ulp of
mpmath's asin over [0, 1], and x > 1 / NaN give NaN like libm.  The GPU build
itself is checked through the eclipse goldens (test_gpu_parity, scalars.npz)."""
import os
import re

import numpy as np
import pytest

mp = pytest.importorskip("mpmath")
HDR = os.path.join(os.path.dirname(__file__), "..", "hb_mcmc_amd", "csrc", "hb_device.hpp")


def _coefs():
    src = open(HDR).read()
    body = src[src.index("double asin01(double x)"):]
    body = body[:body.index("\n}\n")]
    first = re.search(r"double p = ([-0-9.e]+);", body).group(1)
    rest = re.findall(r"p = __builtin_fma\(p, t, ([-0-9.e]+)\);", body)
    return [float(first)] + [float(c) for c in rest]


def _asin01(x, c):
    x = np.asarray(x, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        big = x >= 0.5
        t = np.where(big, (1.0 - x) * 0.5, x * x)
        s = np.where(big, np.sqrt(t), x)
        p = np.full_like(x, c[0])
        for a in c[1:]:
            p = p * t + a
        r = s + (s * t) * p
        return np.where(big, (1.5707963267948966 - 2.0 * r) + 6.123233995736766e-17, r)


def test_asin01_within_3_ulp():
    c = _coefs()
    assert len(c) == 13
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.random(3000), 0.5 + 0.02 * rng.random(500), 1 - rng.random(500) * 1e-9,
                         rng.random(300) * 1e-5, [0.0, 0.5, np.nextafter(0.5, 0.0), 1.0]])
    ys = _asin01(xs, c)
    for x, y in zip(xs, ys):
        ref = mp.asin(mp.mpf(float(x)))
        if ref == 0:
            assert y == 0.0
            continue
        ulp = float(np.spacing(float(ref)))
        assert abs(mp.mpf(float(y)) - ref) <= 3 * ulp, x


def test_asin01_domain():
    c = _coefs()
    out = _asin01(np.array([np.nextafter(1.0, 2.0), 1.5, np.nan]), c)
    assert np.all(np.isnan(out))
