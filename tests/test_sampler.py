"""Bookkeeping parity of the PT-MCMC caller against the REFERENCE sampler's
own trace (tests/golden/sampler_127079833.npz: `HB_MCMC 1200 127079833 0.5021
0`, mcmc_wrapper2.c + likelihood3.c compiled unmodified).

CPU test: the host loop (hb_mcmc_run in libhbmi.so) driven by the oracle's
likelihood -- the oracle is bit-identical to likelihood3.c, so every output
file must match the reference byte for byte.  This checks the sampler logic
(RNG streams, proposals, walls, priors, Hastings, swaps, files); the oracle is
only the likelihood provider of this check, never of the product.

GPU test: the same loop with the GPU likelihood (hb_mcmc CLI): the walker
states/index bookkeeping must still be exact, logL within the stated
tolerance (1e-10 relative).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden

SUF = "127079833_gmag_OMP_0"


def read_outputs(root):
    d = os.path.join(root, "data")
    out = {}
    for key, rel in (("chain", f"chains/chain.{SUF}.dat"), ("logl", f"logL/logL.{SUF}.dat")):
        with open(os.path.join(d, rel), "rb") as fh:
            out[key + "_txt"] = fh.read()
        out[key] = np.loadtxt(os.path.join(d, rel))
    return out


def fixture_files(g):
    return {str(name): bytes(g[f"file{i}"]) for i, name in enumerate(g["file_names"])}


def test_rng_streams_match_reference_algorithm():
    """ran2_parallel seeded <= 0 initialises the shuffle table; > 0 does not."""
    import ctypes as C

    from hb_mcmc_amd import _lib, sampler

    lib = sampler._declare(_lib.lib())
    st = (C.c_byte * 512)()
    C.memset(st, 0, 512)
    C.cast(st, C.POINTER(C.c_long))[0] = 123456789  # idum2
    seed = C.c_long(0)
    v = [lib.hb_ran2_parallel(C.byref(seed), st) for _ in range(3)]
    assert all(0 < x < 1 for x in v) and len(set(v)) == 3


def test_private_rand_is_glibc_rand():
    """The swap draws come from a private copy of glibc's rand(): same sequence
    as libc after srand(seed), for the seeds the CLI uses (NITER) and edges."""
    import ctypes as C

    from hb_mcmc_amd import _lib, sampler

    lib = sampler._declare(_lib.lib())
    libc = C.CDLL("libc.so.6")
    for seed in (0, 1, 1200, 50000, 123456789, 2**31 - 1, 2**31 + 5, 2**32 - 1):
        libc.srand(C.c_uint(seed))
        want = [libc.rand() for _ in range(2000)]
        got = (C.c_int * 2000)()
        lib.hb_rand_stream(seed, 2000, got)
        assert list(got) == want, seed


@pytest.mark.parametrize("skip", [0, 1, 30, 31, 34, 1000, 2 * 4096 * 7 + 3, 10**6])
def test_rand_jump_ahead_equals_sequential(skip):
    """hb_lagfib.hpp: jumping the glibc stream `skip` draws ahead (x^J mod the
    trinomial) gives the same draws as drawing them one by one -- the swap
    schedule of iteration q is built from the stream 2 W q draws on."""
    import ctypes as C

    from hb_mcmc_amd import _lib, sampler

    lib = sampler._declare(_lib.lib())
    for seed in (1, 1200, 2**31 + 5):
        seq = (C.c_int * (skip + 500))()
        lib.hb_rand_stream(seed, skip + 500, seq)
        got = (C.c_int * 500)()
        assert lib.hb_rand_stream_jump(seed, skip, 500, got) == 0
        assert list(got) == list(seq)[skip:], (seed, skip)


@pytest.mark.slow
def test_sampler_bookkeeping_bit_exact_with_oracle_likelihood(oracle, tmp_path):
    from hb_mcmc_amd.sampler import run_mcmc

    g = golden("sampler_127079833.npz")
    t, f, e = g["lc_t"], g["lc_f"], g["lc_e"]
    mag = np.array([1000.0, 1, 1, 1, 1])
    err = np.full(4, 1e15)
    res = run_mcmc(t, f, e, niter=int(g["niter"][0]), run_id="127079833", log10_period=0.5021, run=0,
                   out_root=str(tmp_path), loglik=lambda P: oracle.loglike_batch(t, f, e, P, mag, err, 8),
                   model=lambda p: oracle.light_curve(t, p), nthreads=4)
    out = read_outputs(str(tmp_path))
    assert out["chain_txt"] == bytes(g["chain_txt"])
    assert out["logl_txt"] == bytes(g["logl_txt"])
    for rel, want in fixture_files(g).items():
        with open(os.path.join(str(tmp_path), rel), "rb") as fh:
            assert fh.read() == want, rel
    assert res["loglik_evals"] == 1 + 50 + 1200 * 50  # one batched call per step (+ iteration 0 states)


def run_cli(tmp, niter=1200):
    exe = os.path.join(ROOT, "hb_mcmc_amd", "lib", "hb_mcmc")
    g = stage_input(tmp)
    r = subprocess.run([exe, str(niter), "127079833", "0.5021", "0", "--root", tmp], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stderr
    return g, r.stdout


def stage_input(tmp):
    g = golden("sampler_127079833.npz")
    d = os.path.join(tmp, "data", "lightcurves", "folded_lightcurves")
    os.makedirs(d, exist_ok=True)
    from hb_mcmc_amd.hbio import write_folded_lc

    write_folded_lc(os.path.join(d, "127079833_new.txt"), g["lc_t"], g["lc_f"], g["lc_e"])
    return g


def assert_gpu_run_matches_reference(tmp_path, g):
    """States/bookkeeping exact, logL within 1e-10 relative of the reference trace."""
    out = read_outputs(str(tmp_path))
    ref_chain, ref_logl = g["chain"], g["logl"]
    assert out["chain"].shape == ref_chain.shape and out["logl"].shape == ref_logl.shape
    # iteration column and all 21 parameter columns: exact (same accept/swap decisions)
    assert np.array_equal(out["chain"][:, 0], ref_chain[:, 0])
    assert np.array_equal(out["chain"][:, 2:], ref_chain[:, 2:])
    # logL columns: GPU likelihood vs reference, 1e-10 relative (printed with %.12g)
    for got, want in ((out["chain"][:, 1], ref_chain[:, 1]), (out["logl"][:, 1:], ref_logl[:, 1:])):
        assert np.all(np.abs(got - want) <= 1e-10 * np.maximum(1.0, np.abs(want)))
    # per-slot states of all 50 chains every 100 iterations (%lf): exact
    temps = np.array([np.loadtxt(os.path.join(str(tmp_path), "debug", f"temp_{j}_log.txt")) for j in range(50)])
    assert np.array_equal(temps, g["temps"])
    files = fixture_files(g)
    for rel in (f"data/pars/par.{SUF}.dat", f"data/subpars/subpar.{SUF}.dat"):
        with open(os.path.join(str(tmp_path), rel), "rb") as fh:
            assert fh.read() == files[rel], rel


@pytest.mark.gpu
def test_sampler_bookkeeping_gpu_likelihood(tmp_path):
    g, stdout = run_cli(str(tmp_path))
    assert_gpu_run_matches_reference(tmp_path, g)


@pytest.mark.gpu
def test_reference_sampler_relinked_against_libhbmi(tmp_path):
    """The reference's OWN sampler (src/mcmc_wrapper2.c, unmodified, built by
    `make -C oracle dropin`) linked against libhbmi.so instead of
    likelihood3.c: its 2 x 50 x 1200 scalar loglikelihood() calls, from 25
    OpenMP threads, all run through the drop-in entry point on the GPU."""
    exe = os.path.join(ROOT, "oracle", "_ref", "hb_mcmc_ref_hbmi")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/hb_mcmc_ref_hbmi is built from /root/reference in the development container")
    g = stage_input(str(tmp_path))
    for sub in ("subpars", "pars", "chains", "logL", "log", "lightcurves/mcmc_lightcurves"):
        os.makedirs(os.path.join(str(tmp_path), "data", sub), exist_ok=True)
    os.makedirs(os.path.join(str(tmp_path), "debug"), exist_ok=True)
    r = subprocess.run([exe, "1200", "127079833", "0.5021", "0"], cwd=str(tmp_path),
                       env=dict(os.environ, HBREF_ROOT=str(tmp_path)), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    assert_gpu_run_matches_reference(tmp_path, g)
