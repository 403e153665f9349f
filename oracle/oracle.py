"""ctypes bindings of the parity CHECKERS (test infrastructure only).

Two interchangeable back ends expose the same Python methods:

* ``Oracle()``    -- ``oracle/liboracle.so``, the C restatement of
  likelihood3.c (``oracle/hb_oracle.c``).  Always available (built by
  ``make -C oracle``; gcc exists on the GPU box too).
* ``Reference()`` -- ``oracle/_ref/libref_lik3.so``, the reference
  ``src/likelihood3.c`` compiled unmodified.  Available when it was built in
  the development container (it travels to the GPU box as a binary).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module.  The product package ``hb_mcmc_amd`` never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_D = C.c_double
_PD = C.POINTER(C.c_double)
_L = C.c_long
_I = C.c_int


def _ptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_PD)


def build_oracle() -> str:
    """(Re)build liboracle.so; returns its path."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    return os.path.join(HERE, "liboracle.so")


class _Base:
    # name map: method -> C symbol
    SYM: dict = {}

    def __init__(self, path: str):
        self.path = path
        self.lib = C.CDLL(path)
        s = self._sym
        s("traj").argtypes = [_PD, _PD, _PD, _PD, _PD, _PD, _PD, _I]
        s("get_alpha_beam").restype = _D
        s("get_alpha_beam").argtypes = [_D]
        s("beaming").restype = _D
        s("beaming").argtypes = [_D] * 8
        s("ellipsoidal").restype = _D
        s("ellipsoidal").argtypes = [_D] * 11
        s("reflection").restype = _D
        s("reflection").argtypes = [_D] * 9
        s("eclipse_area").restype = _D
        s("eclipse_area").argtypes = [_D] * 3
        for nm in ("_getT", "_getR", "envelope_Temp", "envelope_Radius", "Eggleton_RL"):
            s(nm).restype = _D
            s(nm).argtypes = [_D]
        s("calc_radii_and_Teffs").argtypes = [_PD, _PD, _PD, _PD, _PD]
        s("calc_mags").argtypes = [_PD, _D, _PD, _PD, _PD, _PD]
        s("calc_light_curve").argtypes = [_PD, _L, _PD, _PD]
        s("RocheOverflow").restype = _I
        s("RocheOverflow").argtypes = [_PD]
        s("loglikelihood").restype = _D
        s("loglikelihood").argtypes = [_PD, _PD, _PD, _L, _PD, _PD, _PD]
        s("remove_median").argtypes = [_PD, _L, _L]
        s("quickSort").argtypes = [_PD, _I, _I]
        s("partition").restype = _D
        s("partition").argtypes = [_PD, _I, _I]
        s("write_lc_to_file").argtypes = [_PD, C.c_char_p]

    def _sym(self, name):
        return getattr(self.lib, self.SYM.get(name, name))

    # -- scalar / vector wrappers (same semantics as the C functions) --
    def traj(self, times, tp):
        times = np.ascontiguousarray(times, dtype=np.float64)
        tp = np.ascontiguousarray(tp, dtype=np.float64)
        n = len(times)
        outs = [np.empty(n) for _ in range(5)]
        self._sym("traj")(_ptr(times), _ptr(tp), *[_ptr(o) for o in outs], n)
        return tuple(outs)  # d, Z1, Z2, rr, ff

    def get_alpha_beam(self, x):
        return self._sym("get_alpha_beam")(x)

    def beaming(self, *a):
        return self._sym("beaming")(*a)

    def ellipsoidal(self, *a):
        return self._sym("ellipsoidal")(*a)

    def reflection(self, *a):
        return self._sym("reflection")(*a)

    def eclipse_area(self, *a):
        return self._sym("eclipse_area")(*a)

    def getT(self, x):
        return self._sym("_getT")(x)

    def getR(self, x):
        return self._sym("_getR")(x)

    def envelope_Temp(self, x):
        return self._sym("envelope_Temp")(x)

    def envelope_Radius(self, x):
        return self._sym("envelope_Radius")(x)

    def eggleton(self, q):
        return self._sym("Eggleton_RL")(q)

    def radii_teffs(self, p):
        p = np.ascontiguousarray(p, dtype=np.float64)
        o = [C.c_double() for _ in range(4)]
        self._sym("calc_radii_and_Teffs")(_ptr(p), *[C.byref(x) for x in o])
        return tuple(x.value for x in o)

    def mags(self, p, dist):
        p = np.ascontiguousarray(p, dtype=np.float64)
        o = [C.c_double() for _ in range(4)]
        self._sym("calc_mags")(_ptr(p), dist, *[C.byref(x) for x in o])
        return tuple(x.value for x in o)

    def roche(self, p):
        p = np.ascontiguousarray(p, dtype=np.float64)
        return int(self._sym("RocheOverflow")(_ptr(p)))

    def light_curve(self, t, p):
        t = np.ascontiguousarray(t, dtype=np.float64)
        p = np.ascontiguousarray(p, dtype=np.float64)
        out = np.empty(len(t))
        self._sym("calc_light_curve")(_ptr(t), len(t), _ptr(p), _ptr(out))
        return out

    def loglike(self, t, f, s, p, mag, magerr):
        """Returns (logL, sigma_after) -- sigma is clamped in place like the reference."""
        t = np.ascontiguousarray(t, dtype=np.float64)
        f = np.ascontiguousarray(f, dtype=np.float64)
        s = np.array(s, dtype=np.float64, copy=True)
        p = np.ascontiguousarray(p, dtype=np.float64)
        mag = np.ascontiguousarray(mag, dtype=np.float64)
        magerr = np.ascontiguousarray(magerr, dtype=np.float64)
        v = self._sym("loglikelihood")(_ptr(t), _ptr(f), _ptr(s), len(t), _ptr(p), _ptr(mag), _ptr(magerr))
        return v, s

    def remove_median(self, a):
        a = np.array(a, dtype=np.float64, copy=True)
        self._sym("remove_median")(_ptr(a), 0, len(a))
        return a

    def quicksort(self, a):
        a = np.array(a, dtype=np.float64, copy=True)
        self._sym("quickSort")(_ptr(a), 0, len(a) - 1)
        return a

    def partition(self, a):
        a = np.array(a, dtype=np.float64, copy=True)
        k = self._sym("partition")(_ptr(a), 0, len(a) - 1)
        return int(k), a

    def write_lc_to_file(self, p, path):
        p = np.ascontiguousarray(p, dtype=np.float64)
        self._sym("write_lc_to_file")(_ptr(p), os.fsencode(path))


class Oracle(_Base):
    SYM = {
        "traj": "orc_orbit",
        "get_alpha_beam": "orc_beam_coeff",
        "beaming": "orc_doppler",
        "ellipsoidal": "orc_tidal",
        "reflection": "orc_irradiation",
        "eclipse_area": "orc_overlap",
        "_getT": "orc_logteff_table",
        "_getR": "orc_logrstar_table",
        "envelope_Temp": "orc_teff_spread",
        "envelope_Radius": "orc_radius_spread",
        "Eggleton_RL": "orc_lobe_fraction",
        "calc_radii_and_Teffs": "orc_stellar",
        "calc_mags": "orc_photometry",
        "calc_light_curve": "orc_light_curve",
        "RocheOverflow": "orc_roche_flag",
        "loglikelihood": "orc_loglike",
        "remove_median": "orc_median_shift",
        "quickSort": "orc_quicksort",
        "partition": "orc_partition",
        "write_lc_to_file": "orc_write_lc_file",
    }

    def __init__(self, path: str | None = None):
        path = path or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build_oracle()
        super().__init__(path)
        L = self.lib
        L.orc_loglike_batch.argtypes = [_PD, _PD, _PD, _L, _PD, _L, _PD, _PD, _PD, _I]
        L.orc_light_curve_batch.argtypes = [_PD, _L, _PD, _L, _PD, _I]
        L.orc_median_value.restype = _D
        L.orc_median_value.argtypes = [_PD, _L]
        L.orc_kepler.argtypes = [_PD, _L, _D, _PD]

    def kepler(self, mean, ecc):
        """The reference's Kepler solve from the mean anomaly (likelihood3.c:
        152-160: start M + 0.85 e sign(sin M), five Newton steps) -- the
        same lines as orc_orbit, which the traj goldens pin."""
        mean = np.ascontiguousarray(mean, dtype=np.float64)
        out = np.empty(len(mean))
        self.lib.orc_kepler(_ptr(mean), len(mean), float(ecc), _ptr(out))
        return out

    def loglike_batch(self, t, f, s, P, mag, magerr, nthreads=0):
        t = np.ascontiguousarray(t, dtype=np.float64)
        f = np.ascontiguousarray(f, dtype=np.float64)
        s = np.array(s, dtype=np.float64, copy=True)
        P = np.ascontiguousarray(P, dtype=np.float64).reshape(-1, 21)
        mag = np.ascontiguousarray(mag, dtype=np.float64)
        magerr = np.ascontiguousarray(magerr, dtype=np.float64)
        out = np.empty(P.shape[0])
        self.lib.orc_loglike_batch(_ptr(t), _ptr(f), _ptr(s), len(t), _ptr(P), P.shape[0], _ptr(mag),
                                   _ptr(magerr), _ptr(out), nthreads)
        return out

    def light_curve_batch(self, t, P, nthreads=0):
        t = np.ascontiguousarray(t, dtype=np.float64)
        P = np.ascontiguousarray(P, dtype=np.float64).reshape(-1, 21)
        out = np.empty((P.shape[0], len(t)))
        self.lib.orc_light_curve_batch(_ptr(t), len(t), _ptr(P), P.shape[0], _ptr(out), nthreads)
        return out

    def median_value(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        return self.lib.orc_median_value(_ptr(a), len(a))


REF_DIR = os.path.join(HERE, "_ref")


def reference_available() -> bool:
    return os.path.exists(os.path.join(REF_DIR, "libref_lik3.so"))


class Reference(_Base):
    """The reference likelihood3.c itself (compiled unmodified)."""

    def __init__(self, path: str | None = None):
        super().__init__(path or os.path.join(REF_DIR, "libref_lik3.so"))
        self.batch = None
        bp = os.path.join(REF_DIR, "libref_batch.so")
        if os.path.exists(bp):
            self.batch = C.CDLL(bp)
            self.batch.ref_loglike_batch.argtypes = [_PD, _PD, _PD, _L, _PD, _L, _PD, _PD, _PD, _I]

    def loglike_batch(self, t, f, s, P, mag, magerr, nthreads=0):
        if self.batch is None:
            raise RuntimeError("libref_batch.so not built")
        t = np.ascontiguousarray(t, dtype=np.float64)
        f = np.ascontiguousarray(f, dtype=np.float64)
        s = np.array(s, dtype=np.float64, copy=True)
        P = np.ascontiguousarray(P, dtype=np.float64).reshape(-1, 21)
        mag = np.ascontiguousarray(mag, dtype=np.float64)
        magerr = np.ascontiguousarray(magerr, dtype=np.float64)
        out = np.empty(P.shape[0])
        self.batch.ref_loglike_batch(_ptr(t), _ptr(f), _ptr(s), len(t), _ptr(P), P.shape[0], _ptr(mag),
                                     _ptr(magerr), _ptr(out), nthreads)
        return out
