"""Drop-in for the reference Cython module ``pyHB`` (src/pyHB.pyx), backed by
libhbmi.so on the GPU.

Same names, argument meanings and error behaviour as pyHB.pyx:31-294:
``lightcurve3``, ``calc_mags``, ``calc_radii_and_Teffs``, ``getR``, ``getT``,
``envelope_Temp``, ``envelope_Radius``, ``parspace`` (+ ``sp2``, ``sp3``),
``likelihood``, ``test_roche_lobe``.

Marshalling quirk kept on purpose: pyHB packs a 22-slot
vector -- [logM1, logM2, logP, e, inc, 0, omega0, T0, rr1, rr2, mu1, tau1,
mu2, tau2, ref1, ref2, exp(b1), exp(b2), aT1, aT2, blend, flux_tune]
(pyHB.pyx:36) -- and hands it to the 21-slot C calc_light_curve
(likelihood3.c:533-578), which therefore reads every slot from 5 on shifted
by one.  The reference module's outputs are reproduced exactly that way
(tests/golden/pyhb.npz was captured from the compiled reference).  Use
``hb_mcmc_amd.likelihood.HBLikelihood`` for the un-shifted 21-slot model.

Batched additions (not in the reference): ``lightcurve3_batch`` and
``likelihood_batch`` evaluate W parameter vectors in one GPU launch.
"""
from __future__ import annotations

import ctypes as C
import sys
import traceback

import numpy as np

from . import _lib

_PD = C.POINTER(C.c_double)

__all__ = ["lightcurve3", "calc_mags", "calc_radii_and_Teffs", "getR", "getT", "envelope_Temp",
           "envelope_Radius", "parspace", "sp2", "sp3", "likelihood", "test_roche_lobe",
           "lightcurve3_batch", "likelihood_batch"]


def _slots22(inpars):
    """The 22-slot vector of pyHB.pyx:36 (beaming factors exponentiated)."""
    (logM1, logM2, logP_day, e, inc, omega0, T0_day, rr1, rr2, mu1, tau1, mu2, tau2, ref1, ref2,
     ln_b1, ln_b2, aT1, aT2, blend, tune) = inpars
    return [logM1, logM2, logP_day, e, inc, 0, omega0, T0_day, rr1, rr2, mu1, tau1, mu2, tau2, ref1, ref2,
            np.exp(ln_b1), np.exp(ln_b2), aT1, aT2, blend, tune]


def _cvec(vals):
    return np.ascontiguousarray(np.asarray(vals, dtype=np.float64))


def lightcurve3(times, inpars):
    """Model light curve at `times` for 21 named parameters (pyHB.pyx:31-69)."""
    cp = _cvec(_slots22(inpars))
    t = _cvec(times)
    out = np.empty(len(t))
    _lib.lib().calc_light_curve(t.ctypes.data_as(_PD), len(t), cp.ctypes.data_as(_PD), out.ctypes.data_as(_PD))
    return out


def lightcurve3_batch(times, P):
    """W x N light curves for a W x 21 array of named parameters (one launch)."""
    from .likelihood import HBLikelihood

    t = _cvec(times)
    P = np.asarray(P, dtype=np.float64).reshape(-1, 21)
    cp = np.array([_slots22(p)[:21] for p in P])  # the C side reads the first 21 slots
    with HBLikelihood(t, np.ones(len(t)), np.ones(len(t))) as L:
        return L.light_curve(cp)


def calc_mags(params, Distance):
    """[G, B-V, V-G, G-T] (pyHB.pyx:71-89); params has 22 entries (incl. ln_noise)."""
    cp = _cvec(_slots22(params[:-1]))
    o = [C.c_double(0.0) for _ in range(4)]
    _lib.lib().calc_mags(cp.ctypes.data_as(_PD), float(Distance), *[C.byref(x) for x in o])
    return [x.value for x in o]


def calc_radii_and_Teffs(params):
    """(R1 [Rsun], R2, Teff1 [K], Teff2) (pyHB.pyx:91-105); 21 named parameters."""
    cp = _cvec(_slots22(params))
    o = [C.c_double(0.0) for _ in range(4)]
    _lib.lib().calc_radii_and_Teffs(cp.ctypes.data_as(_PD), *[C.byref(x) for x in o])
    return o[0].value, o[1].value, o[2].value, o[3].value


def getR(logM):
    return _lib.lib()._getR(float(logM))


def getT(logM):
    return _lib.lib()._getT(float(logM))


def envelope_Temp(logM):
    return _lib.lib().envelope_Temp(float(logM))


def envelope_Radius(logM):
    return _lib.lib().envelope_Radius(float(logM))


class parspace:
    """Named box of parameter ranges with pinning (pyHB.pyx:133-183)."""

    def __init__(self, *args):
        if len(args) % 2 != 0:
            raise ValueError("parspace:Constructor requires arguments in pattern "
                             "('name1',[min,max],'name2',[min,max],...)")
        self.names = list(args[0::2])
        self.mins = np.array([r[0] for r in args[1::2]])
        self.maxs = np.array([r[1] for r in args[1::2]])
        self.N = len(self.names)
        self.live = np.array([True] * self.N)
        self.pinvals = [None] * self.N
        self.idx = {name: i for i, name in enumerate(self.names)}
        self.Nlive = self.N

    def reset_range(self, name, minmax):
        i = self.idx[name]
        if not self.live[i] and (self.pinvals[i] < minmax[0] or self.pinvals[i] > minmax[1]):
            raise ValueError("pinned value is not within range")
        self.mins[i], self.maxs[i] = minmax[0], minmax[1]

    def pin(self, name, value):
        i = self.idx[name]
        if value < self.mins[i] or value > self.maxs[i]:
            print("parspace.pin: Value " + name + " = " + str(value) + "  out of range [" + str(self.mins[i]) + ","
                  + str(self.maxs[i]) + "]")
            return False
        if self.live[i]:
            self.Nlive -= 1
        self.live[i] = False
        self.pinvals[i] = value
        return True

    def get_pars(self, livevals):
        parvals = np.array(self.pinvals)
        parvals[self.live] = livevals
        return parvals

    def live_ranges(self):
        return np.vstack([self.mins[self.live], self.maxs[self.live]]).T

    def live_names(self):
        return [nm for nm, lv in zip(self.names, self.live) if lv]

    def draw_live(self):
        u = np.random.rand(self.Nlive)
        lo, hi = self.mins[self.live], self.maxs[self.live]
        return u * (hi - lo) + lo

    def out_of_bounds(self, pars):
        p = np.array(pars)
        return not np.all((p >= self.mins) & (p <= self.maxs))


sp2 = parspace(  # pyHB.pyx:186-203
    'logM1', [-1.5, 2.0], 'logM2', [-1.5, 2.0], 'logP', [-2.0, 3.0], 'e', [0, 1], 'inc', [0, np.pi],
    'Omega', [-np.pi, np.pi], 'Omega0', [-np.pi, np.pi], 'T0', [-1000, 1000], 'log_rad1_resc', [-2, 2],
    'log_rad2_resc', [-2, 2], 'logTanom', [-0.5, 0.5], 'blend_frac', [0, 1.0], 'logFluxTESS', [-10.0, 10.0],
    'ln_noise_resc', [-0.2, 0.2])

sp3 = parspace(  # pyHB.pyx:205-228
    'logM1', [-1.5, 2.0], 'logM2', [-1.5, 2.0], 'logP', [-2.0, 3.0], 'e', [0, 1], 'inc', [0, np.pi],
    'omega0', [-np.pi, np.pi], 'T0', [-1000, 1000], 'alp_rad1_resc', [-1, 1], 'alp_rad2_resc', [-1, 1],
    'mu_1', [0.12, 0.20], 'tau_1', [0.30, 0.38], 'mu_2', [0.12, 0.20], 'tau_2', [0.30, 0.38],
    'alp_ref_1', [0.8, 1.2], 'alp_ref_2', [0.8, 1.2], 'ln_beam_resc_1', [-0.1, 0.1],
    'ln_beam_resc_2', [-0.1, 0.1], 'alp_Teff_1', [-1, 1], 'alp_Teff_2', [-1, 1], 'blend_frac', [0.0, 1.0],
    'flux_tune', [0.99, 1.01], 'ln_noise_resc', [-0.2, 0.2])

_MINLIKE = -1e18


def likelihood(times, fluxes, errs, pars, lctype=3):
    """Gaussian log-likelihood with a noise rescale (pyHB.pyx:230-252).
    pars = 21 named parameters + ln_noise_resc.  Any exception or NaN -> -1e18."""
    ln_noise_resc = pars[-1]
    pars = pars[:-1]
    try:
        if lctype == 2:
            raise ValueError("lctype=2 no longer supported")
        elif lctype == 3:
            model = lightcurve3(times, pars)
        else:
            raise ValueError('Unknown light curve model type.')
        sigmas = errs * np.exp(ln_noise_resc)
        llike = -np.sum(((fluxes - model) / sigmas) ** 2) / 2 - len(errs) * ln_noise_resc
    except Exception:
        exc_type, exc_value, exc_tb = sys.exc_info()
        print('likelihood exception:')
        traceback.print_exception(exc_type, exc_value, exc_tb, file=sys.stdout)
        llike = _MINLIKE
    if not llike > _MINLIKE:
        llike = _MINLIKE
    return llike


def likelihood_batch(times, fluxes, errs, P, lctype=3):
    """`likelihood` for a W x 22 array in one GPU launch."""
    if lctype != 3:
        raise ValueError("lctype=2 no longer supported" if lctype == 2 else 'Unknown light curve model type.')
    P = np.asarray(P, dtype=np.float64).reshape(-1, 22)
    models = lightcurve3_batch(times, P[:, :21])
    lnr = P[:, 21]
    sig = np.asarray(errs)[None, :] * np.exp(lnr)[:, None]
    ll = -np.sum(((np.asarray(fluxes)[None, :] - models) / sig) ** 2, axis=1) / 2 - len(errs) * lnr
    return np.where(ll > _MINLIKE, ll, _MINLIKE)


def test_roche_lobe(pars, Roche_type='L1', verbose=False):
    """Roche/Hill-radius test statistic (pyHB.pyx:256-294); pars incl. ln_noise.
    Note the reference uses pars[2] (log10 P) directly as P in Kepler's law."""
    M1, M2 = 10 ** pars[0], 10 ** pars[1]
    q = M2 / M1
    P, e = pars[2], pars[3]
    R1, R2, _, _ = calc_radii_and_Teffs(pars[:-1])
    Rsec, Rpri = (R2, R1) if q <= 1 else (R1, R2)
    a = 4.208278 * ((M1 + M2) * P ** 2) ** (1 / 3)
    if Roche_type == 'L1':
        hill = ((q + 2 / 3 + 1 / q) * 3) ** (-1 / 3)
        hill_pri = 1 - hill
    elif Roche_type == 'Eggleton':
        hill = 0.49 / (0.6 + q ** (-2 / 3) * np.log(1 + q ** (1 / 3)))
        hill_pri = 0.49 / (0.6 + q ** (2 / 3) * np.log(1 + q ** (-1 / 3)))
    else:
        raise ValueError('Did not recognize Roche_type="' + str(Roche_type) + '"')
    rperi = a * (1 - e)
    a_sec, a_pri = rperi * hill, rperi * hill_pri
    if verbose:
        print('Roche lobe test: Rsec, RHillsec, Rpri, RHillpri, :', Rsec, a_sec, Rpri, a_pri)
    return max([Rsec / a_sec, Rpri / a_pri])
