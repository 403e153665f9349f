"""hb_mcmc_amd.pyHB against outputs of the REFERENCE Cython module pyHB
(compiled from src/pyHB.pyx; captured in tests/golden/pyhb.npz), and
INTEGRATION.md Option B (the reference pyHB.pyx relinked against libhbmi.so)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, golden

REF_PYX = "/root/reference/src/pyHB.pyx"


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


def test_option_b_reference_pyhb_relinked_against_libhbmi(tmp_path):
    """INTEGRATION.md section 4, Option B: the reference's pyHB.pyx, unmodified,
    compiled against include/hbmi.h (oracle/pyhb_hbmi/likelihood3.pxd) and
    linked to libhbmi.so.  Built here in a temporary directory (the module
    embeds the reference's source, so it never travels to the GPU box): it
    imports, its seven likelihood3 entry points resolve from libhbmi.so, and
    without a GPU a call fails loudly instead of falling back to the CPU."""
    if not os.path.exists(REF_PYX):
        pytest.skip("the reference sources exist in the development container only")
    out = str(tmp_path / "pyhb_hbmi")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "pyhb_hbmi", f"PYHB_HBMI_DIR={out}"],
                   check=True, capture_output=True, timeout=600)
    so = [f for f in os.listdir(out) if f.startswith("pyHB") and f.endswith(".so")]
    assert len(so) == 1
    und = subprocess.run(["nm", "-D", "--undefined-only", os.path.join(out, so[0])], capture_output=True,
                         text=True, check=True).stdout.split()
    entry = ["calc_light_curve", "calc_radii_and_Teffs", "calc_mags", "_getT", "_getR", "envelope_Radius",
             "envelope_Temp"]
    assert all(e in und for e in entry)
    libs = subprocess.run(["ldd", os.path.join(out, so[0])], capture_output=True, text=True, check=True).stdout
    assert os.path.join(ROOT, "hb_mcmc_amd", "lib", "libhbmi.so") in libs
    probe = ("import sys; sys.path.insert(0, %r); import pyHB; "
             "names = ['lightcurve3', 'calc_mags', 'calc_radii_and_Teffs', 'getR', 'getT', 'envelope_Temp', "
             "'envelope_Radius', 'likelihood', 'parspace', 'test_roche_lobe']; "
             "print('missing', [n for n in names if not hasattr(pyHB, n)], flush=True)" % out)
    r = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "missing []" in r.stdout, r.stderr[-2000:]
    from hb_mcmc_amd import _lib

    if not _lib.device_available():
        r = subprocess.run([sys.executable, "-c", probe + "; pyHB.getR(0.1)"], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode != 0 and "no HIP device" in r.stderr
