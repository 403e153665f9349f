"""Why the cold path's series Kepler start pays (hb_device.hpp cold_start_k,
|e| <= kSeriesEmax = 0.25), in numpy float64: Newton steps to the kernel's
stopping rule (predicted next correction e d^2 / (2 (1 - e cos E)) <= 2^-52),
as the maximum over a wave of 64 consecutive mean anomalies, from the
reference's start E0 = M + 0.85 e sign(sin M) (likelihood3.c:155-157) and from
the Lagrange series of Kepler's equation to third, fourth and fifth order; the
start's worst error and the converged root's distance to the true root; and
the factored fifth-order form the kernel evaluates against the textbook sum.

    python scripts/kepler_series.py
"""
import numpy as np


def newton_steps(M, E, e, maxit=8):
    n = np.zeros(M.shape, int)
    done = np.zeros(M.shape, bool)
    for it in range(maxit):
        den = 1 - e * np.cos(E)
        d = ((E - e * np.sin(E)) - M) / den
        E = np.where(done, E, E - d)
        n = np.where(done, n, it + 1)
        done |= e * d * d <= 2.0 ** -51 * den
    return n, E


def root(M, e):
    E = M + 0.85 * e * np.sign(np.sin(M))
    for _ in range(60):
        E = E - ((E - e * np.sin(E)) - M) / (1 - e * np.cos(E))
    return E


def series(M, e, order):
    s = np.sin(M)
    d = e * s
    if order >= 2:
        d = d + e ** 2 / 2 * np.sin(2 * M)
    if order >= 3:
        d = d + e ** 3 / 8 * (3 * np.sin(3 * M) - s)
    if order >= 4:
        d = d + e ** 4 / 6 * (2 * np.sin(4 * M) - np.sin(2 * M))
    if order >= 5:
        d = d + e ** 5 / 384 * (125 * np.sin(5 * M) - 81 * np.sin(3 * M) + 2 * s)
    return M + d


def kernel_form(M, e):  # hb_device.hpp cold_start_k
    s, c = np.sin(M), np.cos(M)
    x = s * s
    a = (e ** 2 + e ** 4) + x * (-8 / 3 * e ** 4)
    b = (e + e ** 3 + e ** 5) + x * (-(1.5 * e ** 3 + 17 / 3 * e ** 5) + x * (125 / 24 * e ** 5))
    return M + s * (c * a + b)


M = np.linspace(-np.pi, np.pi, 64 * 2000, endpoint=False)
print("e | wave steps (mean, max) from: reference start, series order 3, 4, 5 | start error of order 5 | "
      "|converged - root| | |kernel form - order-5 sum|")
for e in (0.05, 0.1, 0.2, 0.226, 0.25, 0.3, 0.4, 0.5):
    R = root(M, e)
    row = []
    for E0 in (M + 0.85 * e * np.sign(np.sin(M)), series(M, e, 3), series(M, e, 4), series(M, e, 5)):
        n, E = newton_steps(M, E0, e)
        w = n.reshape(-1, 64).max(1)
        row.append(f"{w.mean():.2f}/{w.max()}")
        err = np.abs(E - R).max()
    print(f"{e:5.3f} | {' '.join(row)} | {np.abs(series(M, e, 5) - R).max():.1e} | {err:.1e} | "
          f"{np.abs(kernel_form(M, e) - series(M, e, 5)).max():.1e}")
