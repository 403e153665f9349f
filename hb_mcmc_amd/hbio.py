"""Readers/writers of the reference's file formats.

* folded light curve ``<TIC>_new.txt``: first line N, then N lines
  ``t<TAB>flux<TAB>err`` (src/README.txt:13-19; reader
  src/mcmc_wrapper2.c:257-298);
* magnitude file ``<TIC>.txt``: distance, then 4 lines ``value<TAB>error``
  for G, B-V, V-G, G-T (src/README.txt:21-28; reader mcmc_wrapper2.c:302-328);
  when absent the reference falls back to D=1000, mags=1, errors=1e15.
* periods table ``periods.txt``: ``TIC<TAB>period_days<TAB>flag``;
* colour/photometry catalogue ``data/color_mag/cp_data_4-21-2022.csv`` (written
  by src/tic_processing.py:268-300 make_cp_data, one row per TIC: dist, the
  dereddened Gmag0 and colours BmV0/VmG0/GmT0 with their errors, ...):
  read_cp_data + cp_mag_data give each target's (mag_data[5], magerr[4]).
"""
from __future__ import annotations

import csv
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


def write_mag_file(path: str, mag, err) -> None:
    """The magnitude file mcmc_wrapper2.c:302-315 reads (src/README.txt:21-28)."""
    with open(path, "w") as fh:
        fh.write(f"{float(mag[0])!r}\n")
        for k in range(4):
            fh.write(f"{float(mag[k + 1])!r}\t{float(err[k])!r}\n")


def read_cp_data(path: str) -> dict:
    """cp_data CSV -> {TIC_ID (str): {column: float or None, 'flags': str}}.
    Empty fields are None (tic_processing.py:140-222 leaves unknown values
    unset)."""
    out = {}
    with open(path, newline="") as fh:
        for row in csv.DictReader(fh):
            rec = {}
            for k, v in row.items():
                if k in ("TIC_ID", "flags"):
                    continue
                v = (v or "").strip()
                rec[k] = float(v) if v else None
            rec["flags"] = row.get("flags", "")
            out[row["TIC_ID"].strip()] = rec
    return out


def cp_mag_data(rec: dict | None):
    """(mag_data[5], magerr[4]) = ({dist, Gmag0, BmV0, VmG0, GmT0}, their
    errors) for one cp_data record.  Missing values take the fallbacks the
    reference's own mag-file writer uses (src/helpful_functions.py:377-420):
    distance 1000 pc; G 10 with error 1e4; a colour 0 with error 1e3; a known
    value without an error gets error 1.  rec None: the reader's fallback for
    an absent mag file (mcmc_wrapper2.c:321-327)."""
    if rec is None:
        return MAG_DEFAULT.copy(), MAGERR_DEFAULT.copy()

    def val(k):
        v = rec.get(k)
        return None if v is None or v != v else v

    dist = val("dist")
    mag = np.empty(5)
    err = np.empty(4)
    mag[0] = dist if dist else 1000.0
    g = val("Gmag0")
    if g is None:
        mag[1], err[0] = 10.0, 10000.0
    else:
        ge = val("Gmag0_e")
        mag[1], err[0] = g, (ge if ge else 1.0)
    for k, col in enumerate(("BmV0", "VmG0", "GmT0")):
        c = val(col)
        if c is None:
            mag[2 + k], err[1 + k] = 0.0, 1000.0
        else:
            ce = val(col + "_e")
            mag[2 + k], err[1 + k] = c, (ce if ce else 1.0)
    return mag, err


DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def load_folded_catalog(npz: str | None = None, cp_csv: str | None = None):
    """The reference's 111 folded light curves (data/folded_catalog.npz, packed
    by scripts/pack_catalog.py from data/lightcurves/folded_lightcurves/ and
    periods.txt) with each target's magnitude block from the cp_data CSV.
    Returns a list of dicts: tic, name, period [d], t, flux, sigma, mag, magerr."""
    z = np.load(npz or os.path.join(DATA_DIR, "folded_catalog.npz"), allow_pickle=False)
    cp = read_cp_data(cp_csv or os.path.join(DATA_DIR, "cp_data_4-21-2022.csv"))
    out, o = [], 0
    for k, nk in enumerate(z["n"]):
        nk = int(nk)
        tic = str(z["tics"][k])
        mag, err = cp_mag_data(cp.get(tic))
        out.append({"tic": tic, "name": str(z["names"][k]), "period": float(z["periods"][k]),
                    "t": z["t"][o:o + nk].copy(), "flux": z["f"][o:o + nk].copy(),
                    "sigma": z["e"][o:o + nk].copy(), "mag": mag, "magerr": err})
        o += nk
    return out
