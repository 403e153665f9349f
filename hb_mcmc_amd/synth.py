"""Synthetic workloads of SURVEY.md section 8(d) (deterministic, numpy PCG64).

* truth vector ``THETA_STAR`` -- the reference's own test pin,
  src/test_likelihoods.c:33-36 (P = 10**0.315687018 ~ 2.069 d);
* cadences t_i = 2 P i / N (two phases, like the doubled folded files);
* sigma_i = 1e-3, flux = model(THETA_STAR) + sigma * n_i, n_i ~ N(0, 1);
* walkers theta_w = THETA_STAR + 0.1 * sigma_prop * z_w reflected into the
  set_limits prior box (likelihood3.c:986-1121), slot 2 (log P) fixed, with a
  fraction pushed into Roche-lobe overflow (e -> 0.9x, logL = -5e14).
* prior-spread walkers (``prior_walkers``): uniform over the set_limits box
  like the reference's random initial state (mcmc_wrapper2.c:236-252) -- the
  spread the sampler's hot rungs keep: e over [0, 1), cold-path and Roche
  walkers.
* mag_data = {1000, 1, 1, 1, 1}, magerr = 1e15 (mcmc_wrapper2.c:321-327).
"""
from __future__ import annotations

import numpy as np

NPARS = 21

THETA_STAR = np.array([
    0.300918167925, 0.201073240382, 0.315687018, 0.226228332961, 1.43483081695, 2.39254328279,
    1.53065288845, -2.45048204944, -0.0111151536831, 0.17004110046, 0.334086604211, 0.155971855936,
    0.339246868468, 0.94581378228, 0.824791381832, -0.0140470354976, -0.0368550857758, 0.41323817757,
    0.547024296055, 0.308828039741, 1.00029951763])

# proposal widths after the no-colour override (likelihood3.c:1135-1179)
SIGMA_PROP = np.array([1e-1, 1e-1, 1e-8, 1e-2, 1e-2, 1e-2, 1e-3, 1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e-1,
                       1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e-1, 1e-3, 1e-5])

MAG_DEFAULT = np.array([1000.0, 1.0, 1.0, 1.0, 1.0])
MAGERR_DEFAULT = np.array([1e15, 1e15, 1e15, 1e15])


def prior_box(lc_period: float):
    """(lo, hi, kind) per slot; kind 1 = reflecting wall, 2 = periodic, 0 = open.
    Mirrors set_limits (likelihood3.c:986-1121) incl. its quirk that e has no
    upper wall (limited[3].hi = 0.99 != 1)."""
    pi = np.pi
    lo = np.array([-1.5, -1.5, -2.0, 0.0, 0.0, -pi, 0.0, -5, -5, 0.12, 0.3, 0.12, 0.3, 0.5, 0.5,
                   -0.3, -0.3, -5, -5, 0.0, 0.99])
    hi = np.array([2.0, 2.0, 3.0, 1.0, pi, pi, lc_period, 5, 5, 0.20, 0.38, 0.20, 0.38, 1.5, 1.5,
                   0.3, 0.3, 5, 5, 1.0, 1.01])
    kind_lo = np.ones(NPARS, dtype=int)
    kind_hi = np.ones(NPARS, dtype=int)
    kind_lo[5] = kind_hi[5] = 2
    kind_hi[3] = 0
    return lo, hi, kind_lo, kind_hi


def cadences(n: int, period_days: float | None = None) -> np.ndarray:
    p = 10.0 ** THETA_STAR[2] if period_days is None else period_days
    return 2.0 * p * np.arange(n, dtype=np.float64) / n


def noise(n: int, seed: int = 20260101) -> np.ndarray:
    return np.random.Generator(np.random.PCG64(seed)).standard_normal(n)


def reflect_into_box(x: np.ndarray, lc_period: float) -> np.ndarray:
    lo, hi, klo, khi = prior_box(lc_period)
    y = x.copy()
    for i in range(NPARS):
        col = y[..., i]
        for _ in range(64):
            m_lo = (klo[i] == 1) & (col < lo[i])
            m_hi = (khi[i] == 1) & (col > hi[i])
            if not (m_lo.any() or m_hi.any()):
                break
            col = np.where(m_lo, 2 * lo[i] - col, col)
            col = np.where(m_hi, 2 * hi[i] - col, col)
        if klo[i] == 2:
            col = lo[i] + np.mod(col - lo[i], hi[i] - lo[i])
        y[..., i] = col
    return y


def walkers(w: int, seed: int = 7, roche_frac: float = 0.05, scale: float = 0.1,
            theta: np.ndarray | None = None) -> np.ndarray:
    """W x 21 walker parameter vectors around the truth."""
    th = THETA_STAR if theta is None else np.asarray(theta, dtype=np.float64)
    g = np.random.Generator(np.random.PCG64(seed))
    lc_period = 10.0 ** th[2]
    z = g.standard_normal((w, NPARS))
    x = th[None, :] + scale * SIGMA_PROP[None, :] * z
    x = reflect_into_box(x, lc_period)
    x[:, 2] = th[2]
    x[:, 6] = np.fmod(x[:, 6], lc_period)
    nro = int(round(roche_frac * w))
    if nro:
        idx = g.choice(w, size=nro, replace=False)
        x[idx, 3] = 0.9 + 0.09 * g.random(nro)  # tight periastron -> Roche overflow
    return np.ascontiguousarray(x)


def prior_walkers(w: int, seed: int = 11, theta: np.ndarray | None = None) -> np.ndarray:
    """W x 21 walkers drawn uniformly from the set_limits box, slot 2 = the
    light curve's log P and slot 6 folded into [0, P), as the reference's
    random initial state (mcmc_wrapper2.c:236-252: x = lo + u (hi - lo))."""
    th = THETA_STAR if theta is None else np.asarray(theta, dtype=np.float64)
    lc_period = 10.0 ** th[2]
    lo, hi, _, _ = prior_box(lc_period)
    u = np.random.Generator(np.random.PCG64(seed)).random((w, NPARS))
    x = lo[None, :] + u * (hi - lo)[None, :]
    x[:, 2] = th[2]
    x[:, 6] = np.fmod(x[:, 6], lc_period)
    return np.ascontiguousarray(x)


def dataset(n: int, model_fn, seed: int = 20260101, sigma: float = 1e-3):
    """(t, flux, sigma) with flux = model_fn(t, THETA_STAR) + sigma * n."""
    t = cadences(n)
    s = np.full(n, sigma)
    f = np.asarray(model_fn(t, THETA_STAR), dtype=np.float64) + s * noise(n, seed)
    return t, f, s
