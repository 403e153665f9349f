"""hb_mcmc_amd.pyHB against outputs of the REFERENCE Cython module pyHB
(compiled from src/pyHB.pyx; captured in tests/golden/pyhb.npz)."""
import numpy as np
import pytest

from conftest import golden


def test_parspace_boxes_and_pinning():
    from hb_mcmc_amd import pyHB

    g = golden("pyhb.npz")
    assert list(pyHB.sp3.names) == [str(x) for x in g["sp3_names"]]
    assert list(pyHB.sp2.names) == [str(x) for x in g["sp2_names"]]
    assert np.array_equal(np.c_[pyHB.sp3.mins, pyHB.sp3.maxs], g["sp3"])
    assert np.array_equal(np.c_[pyHB.sp2.mins, pyHB.sp2.maxs], g["sp2"])
    sp = pyHB.parspace("a", [0, 1], "b", [-1, 1], "c", [2, 3])
    assert sp.pin("b", 0.5) and not sp.pin("a", 7.0)
    assert sp.Nlive == 2 and sp.live_names() == ["a", "c"]
    assert np.array_equal(sp.get_pars([0.25, 2.5]), [0.25, 0.5, 2.5])
    assert sp.out_of_bounds([0.1, 0.5, 4.0]) and not sp.out_of_bounds([0.1, 0.5, 2.1])
    with pytest.raises(ValueError):
        sp.reset_range("b", [0.6, 0.9])
    with pytest.raises(ValueError):
        pyHB.parspace("a", [0, 1], "b")
    d = sp.draw_live()
    assert d.shape == (2,) and 0 <= d[0] <= 1 and 2 <= d[1] <= 3


def test_likelihood_error_path_returns_minlike():
    from hb_mcmc_amd import pyHB

    assert pyHB.likelihood(np.arange(3.0), np.ones(3), np.ones(3), [0.0] * 22, lctype=2) == -1e18


@pytest.mark.gpu
def test_pyhb_surface_matches_reference_module(hbmi):
    from hb_mcmc_amd import pyHB

    g = golden("pyhb.npz")
    t, P = g["t"], g["params"]
    lc = np.array([pyHB.lightcurve3(t, list(p)) for p in P])
    assert np.abs(lc - g["lc3"]).max() <= 1e-12
    assert np.abs(pyHB.lightcurve3_batch(t, P) - g["lc3"]).max() <= 1e-12
    like = np.array([pyHB.likelihood(t, g["f"], g["errs"], list(p) + [r]) for p, r in zip(P, g["lnr"])])
    assert np.all(np.abs(like - g["like"]) <= 1e-10 * np.maximum(1, np.abs(g["like"])))
    lb = pyHB.likelihood_batch(t, g["f"], g["errs"], np.c_[P, g["lnr"]])
    assert np.all(np.abs(lb - g["like"]) <= 1e-10 * np.maximum(1, np.abs(g["like"])))
    mags = np.array([pyHB.calc_mags(list(p) + [0.0], 300.0) for p in P])
    assert np.allclose(mags, g["mags"], rtol=1e-12, atol=1e-12)
    radii = np.array([pyHB.calc_radii_and_Teffs(list(p)) for p in P])
    assert np.allclose(radii, g["radii"], rtol=1e-12, atol=0)
    gr = np.array([[pyHB.getR(x), pyHB.getT(x), pyHB.envelope_Temp(x), pyHB.envelope_Radius(x)] for x in g["lm"]])
    assert np.allclose(gr, g["getR_getT_envT_envR"], rtol=1e-12, atol=1e-15)
    rl = np.array([[pyHB.test_roche_lobe(list(p) + [0.0]), pyHB.test_roche_lobe(list(p) + [0.0], "Eggleton")]
                   for p in P])
    assert np.allclose(rl, g["roche"], rtol=1e-12, atol=0)
