"""Host-side logic that needs no GPU: workload generator, file formats."""
import os

import numpy as np

from conftest import golden
from hb_mcmc_amd import hbio, synth


def test_walkers_deterministic_and_in_box():
    a, b = synth.walkers(512, seed=3), synth.walkers(512, seed=3)
    assert np.array_equal(a, b)
    lo, hi, klo, khi = synth.prior_box(10 ** synth.THETA_STAR[2])
    inside = [(klo[i] != 1 or (a[:, i] >= lo[i]).all()) and (khi[i] != 1 or (a[:, i] <= hi[i]).all())
              for i in range(21)]
    assert all(inside)
    assert (a[:, 2] == synth.THETA_STAR[2]).all()


def test_prior_box_matches_set_limits():
    g = golden("limits.npz")
    lo, hi, klo, khi = synth.prior_box(float(g["lc_period"][0]))
    assert np.array_equal(lo, g["limits"][:, 0]) and np.array_equal(hi, g["limits"][:, 1])
    assert np.array_equal(klo, g["limited"][:, 0].astype(int))
    # e's upper flag is 0.99 in the reference: no wall (kind 0 here)
    assert g["limited"][3, 1] == 0.99 and khi[3] == 0


def test_folded_lc_roundtrip(tmp_path):
    t = np.linspace(0, 1, 17)
    f = 1 + 0.001 * np.sin(t)
    e = np.full(17, 3e-4)
    p = os.path.join(tmp_path, "x_new.txt")
    hbio.write_folded_lc(p, t, f, e)
    t2, f2, e2 = hbio.read_folded_lc(p)
    assert np.array_equal(t, t2) and np.array_equal(f, f2) and np.array_equal(e, e2)


def test_mag_file_fallback(tmp_path):
    mag, err = hbio.read_mag_file(os.path.join(tmp_path, "missing.txt"))
    assert np.array_equal(mag, [1000, 1, 1, 1, 1]) and np.array_equal(err, [1e15] * 4)
    p = os.path.join(tmp_path, "m.txt")
    with open(p, "w") as fh:
        fh.write("512.5\n10.1\t0.01\n0.3\t0.02\n0.1\t0.03\n0.2\t0.04\n")
    mag, err = hbio.read_mag_file(p)
    assert np.array_equal(mag, [512.5, 10.1, 0.3, 0.1, 0.2]) and np.array_equal(err, [0.01, 0.02, 0.03, 0.04])


def test_real_fixture_is_reference_data():
    g = golden("lc_real231937440.npz")
    assert g["t"].shape == (883,) and g["t"][0] == 0.001164 and g["f"][0] == 0.999987
