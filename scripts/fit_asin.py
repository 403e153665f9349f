"""Coefficients of the eclipse kernels' asin (hb_device.hpp asin01): a
degree-12 Chebyshev fit (mpmath, 50 digits) of P(t) = (asin(s) - s) / (s t),
s = sqrt(t), on [0, 1/4], so that asin(s) = s + s t P(t).  Prints the
coefficients (highest degree first) and the largest error of the float64
evaluation against mpmath's asin over [0, 1] in units in the last place."""
import mpmath as mp
import numpy as np

mp.mp.dps = 50


def f(t):
    s = mp.sqrt(t)
    return (mp.asin(s) - s) / (s * t)


c, err = mp.chebyfit(f, [mp.mpf(0), mp.mpf(1) / 4], 13, error=True)
cd = [float(x) for x in c]
print("fit error", mp.nstr(err, 4))
for x in cd:
    print(repr(x))


def asin01(x):  # the device evaluation order (fma -> mul + add here: within an ulp of it)
    big = x >= 0.5
    t = np.where(big, (1.0 - x) * 0.5, x * x)
    s = np.where(big, np.sqrt(np.maximum(t, 0.0)), x)
    p = np.full_like(x, cd[0])
    for a in cd[1:]:
        p = p * t + a
    r = s + (s * t) * p
    return np.where(big, (1.5707963267948966 - 2.0 * r) + 6.123233995736766e-17, r)


rng = np.random.default_rng(1)
xs = np.concatenate([rng.random(20000), 1 - rng.random(5000) * 1e-6, rng.random(5000) * 1e-4,
                     np.array([0.5, np.nextafter(0.5, 0), 1.0, 0.0, 0.25])])
ys = asin01(xs)
worst, wx = 0, None
for x, y in zip(xs, ys):
    ref = mp.asin(mp.mpf(float(x)))
    if ref == 0:
        continue
    u = abs(mp.mpf(float(y)) - ref) / mp.mpf(float(np.spacing(float(ref))))
    if u > worst:
        worst, wx = u, x
print("max ulp error", mp.nstr(worst, 4), "at", wx)
