"""Readers/writers of the reference's file formats.

* folded light curve ``<TIC>_new.txt``: first line N, then N lines
  ``t<TAB>flux<TAB>err`` (src/README.txt:13-19; reader
  src/mcmc_wrapper2.c:257-298);
* magnitude file ``<TIC>.txt``: distance, then 4 lines ``value<TAB>error``
  for G, B-V, V-G, G-T (src/README.txt:21-28; reader mcmc_wrapper2.c:302-328);
  when absent the reference falls back to D=1000, mags=1, errors=1e15.
* periods table ``periods.txt``: ``TIC<TAB>period_days<TAB>flag``.
"""
from __future__ import annotations

import os

import numpy as np

from .synth import MAG_DEFAULT, MAGERR_DEFAULT


def read_folded_lc(path: str):
    """Returns (t, flux, err) as float64 arrays (N from the header line)."""
    with open(path) as fh:
        n = int(fh.readline().split()[0])
        rows = np.loadtxt(fh, dtype=np.float64, ndmin=2, max_rows=n)
    if rows.shape[0] != n:
        raise ValueError(f"{path}: header says {n} rows, found {rows.shape[0]}")
    return (np.ascontiguousarray(rows[:, 0]), np.ascontiguousarray(rows[:, 1]),
            np.ascontiguousarray(rows[:, 2]))


def write_folded_lc(path: str, t, f, e):
    with open(path, "w") as fh:
        fh.write(f"{len(t)}\n")
        for a, b, c in zip(t, f, e):
            fh.write(f"{float(a)!r}\t{float(b)!r}\t{float(c)!r}\n")


def read_mag_file(path: str | None):
    """Returns (mag_data[5], magerr[4]); reference fallback when missing."""
    if path is None or not os.path.exists(path):
        return MAG_DEFAULT.copy(), MAGERR_DEFAULT.copy()
    with open(path) as fh:
        vals = fh.read().split()
    d = float(vals[0])
    rest = [float(v) for v in vals[1:9]]
    mag = np.array([d, rest[0], rest[2], rest[4], rest[6]])
    err = np.array([rest[1], rest[3], rest[5], rest[7]])
    return mag, err


def read_periods(path: str) -> dict:
    out = {}
    with open(path) as fh:
        for line in fh:
            parts = line.split()
            if len(parts) >= 2:
                out[parts[0]] = float(parts[1])
    return out
