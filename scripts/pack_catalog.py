"""Pack the reference's 111 folded light curves (data/lightcurves/
folded_lightcurves/*, read as mcmc_wrapper2.c:257-298 reads them) and their
periods (data/lightcurves/periods.txt) into data/folded_catalog.npz, the
real-target part of the C5 catalog bench (bench.py --config C5) and of the
catalog GPU test.  Data only; run in the development container:

    python scripts/pack_catalog.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hb_mcmc_amd.hbio import read_folded_lc, read_periods  # noqa: E402

REF = os.environ.get("HB_REFERENCE", "/root/reference")
D = os.path.join(REF, "data", "lightcurves", "folded_lightcurves")
per = read_periods(os.path.join(REF, "data", "lightcurves", "periods.txt"))
names, tics, periods, n, t, f, e = [], [], [], [], [], [], []
for fn in sorted(os.listdir(D)):
    tt, ff, ee = read_folded_lc(os.path.join(D, fn))
    tic = fn.replace("_new.txt", "")
    names.append(fn)
    tics.append(tic)
    periods.append(per[tic])
    n.append(len(tt))
    t.append(tt)
    f.append(ff)
    e.append(ee)
out = os.path.join(ROOT, "data", "folded_catalog.npz")
np.savez_compressed(out, names=np.array(names), tics=np.array(tics), periods=np.array(periods),
                    n=np.array(n), t=np.concatenate(t), f=np.concatenate(f), e=np.concatenate(e))
print(f"wrote {out}: {len(names)} light curves, N in [{min(n)}, {max(n)}], {os.path.getsize(out)} B")
