"""Shader cycles of the device sampler's wall folds (hbwall::apply_wall) per
value, one wave per value (64 lanes folding the same value, no other wave on
its SIMD): values at 2^k ranges outside each wall range of the sampler
(set_limits), both sides.  Prints JSON: range, side, k, value, cycles.  The
fold / pass counts of the same values come from the CPU.

    python scripts/wall_probe.py > gpurun_out/wall_probe.json
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hb_mcmc_amd import _lib  # noqa: E402

RANGES = [(0.3, 0.38), (0.12, 0.2), (0.5, 1.5), (-0.3, 0.3), (0.0, 0.99), (-1.5, 2.0), (-5.0, 5.0)]
lib = _lib.lib()
f = lib.hbx_wall_probe
PD = C.POINTER(C.c_double)
f.argtypes = [PD, PD, PD, C.c_long, PD, C.POINTER(C.c_longlong)]
f.restype = C.c_int
rows, vals, los, his = [], [], [], []
rng = np.random.default_rng(5)
for lo, hi in RANGES:
    w = hi - lo
    for side in (-1, 1):
        for k2 in range(0, 37):
            k = k2 / 2.0
            d = w * (2.0 ** k) * (1.0 + 0.37 * rng.random())
            v = hi + d if side > 0 else lo - d
            rows.append({"lo": lo, "hi": hi, "side": side, "k": k, "v": v})
            vals += [v] * 64
            los += [lo] * 64
            his += [hi] * 64
v = np.array(vals)
lo = np.array(los)
hi = np.array(his)
out = np.empty_like(v)
cyc = np.empty(len(rows), dtype=np.int64)
for rep in range(3):  # the last repetition is kept (clock ramped)
    rc = f(v.ctypes.data_as(PD), lo.ctypes.data_as(PD), hi.ctypes.data_as(PD), len(v), out.ctypes.data_as(PD),
           cyc.ctypes.data_as(C.POINTER(C.c_longlong)))
    assert rc == 0, _lib.last_error()
for r, c, o in zip(rows, cyc, out[::64]):
    r["cycles"] = int(c)
    r["out"] = float(o)
print(json.dumps(rows))
