"""Catalog-sweep mode (config C5, hb_mcmc_amd/catalog.py, include/hbmi.h
hb_catalog_*): many targets on one GPU, every size class in one eval launch.

CPU: the lockstep multi-target sampler driven by the oracle likelihood writes,
for every target, exactly the files the single-target sampler writes for it
alone (byte for byte); targets are dealt over ranks by cadence count.
GPU: the batched catalog equals per-target contexts bit for bit (within
the oracle tolerance for N = 1025..1280, where the catalog runs a pair of
waves and a lone context one wave: other chain starts, chi^2 summed in
another order) and the oracle within 1e-10
(every size class N = 2..2048, zero-walker targets, per-target magnitude
data); the GPU sweep equals the single-target GPU runs.
"""
import filecmp
import os

import numpy as np
import pytest

from conftest import golden

LOGL_RTOL = 1e-10


def synth_target(n, seed, orc, gmag=None):
    from hb_mcmc_amd import synth

    t, f, s = synth.dataset(n, orc.light_curve)
    rng = np.random.default_rng(seed)
    f = f + 1e-4 * rng.standard_normal(n)
    if gmag is None:
        return (t, f, s)
    return (t, f, s, np.array([850.0, gmag, 1, 1, 1]), np.array([0.02, 1e15, 1e15, 1e15]))


def tree_files(root):
    out = []
    for d, _, fs in os.walk(root):
        out += [os.path.relpath(os.path.join(d, f), root) for f in fs]
    return sorted(out)


def test_deal_targets_balances_cadences():
    from hb_mcmc_amd.catalog import deal_targets

    rng = np.random.default_rng(3)
    ncad = rng.integers(82, 1862, 256)
    for world in (1, 2, 3, 8):
        owner = deal_targets(ncad, world)
        load = np.bincount(owner, weights=ncad, minlength=world)
        assert len(owner) == 256 and set(owner) <= set(range(world))
        assert load.max() - load.min() <= ncad.max()


def test_catalog_sweep_equals_single_target_runs(tmp_path, oracle):
    from hb_mcmc_amd.catalog import run_catalog
    from hb_mcmc_amd.sampler import run_mcmc

    g = golden("sampler_127079833.npz")
    targets = [(g["lc_t"], g["lc_f"], g["lc_e"]), synth_target(300, 1, oracle), synth_target(97, 2, oracle)]
    ids, periods = ["127079833", "9001", "9002"], [0.5021, 0.3157, 0.3157]
    mag, err = np.array([1000.0, 1, 1, 1, 1]), np.full(4, 1e15)

    def ll_multi(P, walkers):
        out, o = [], 0
        for k, w in enumerate(walkers):
            t, f, s = targets[k]
            out.append(oracle.loglike_batch(t, f, s, P[o:o + w], mag, err, 1) if w else np.empty(0))
            o += w
        return np.concatenate(out)

    kw = dict(niter=260, nchains=9, npast=20, run=2)
    res = run_catalog(targets, run_ids=ids, log10_periods=periods, out_root=str(tmp_path / "cat"), nthreads=2,
                      loglik_multi=ll_multi, model=lambda k, p: oracle.light_curve(targets[k][0], p), **kw)
    for k in range(3):
        t, f, s = targets[k]
        root = str(tmp_path / "one" / ids[k])
        ref = run_mcmc(t, f, s, run_id=ids[k], log10_period=periods[k], out_root=root, nthreads=2,
                       loglik=lambda P, t=t, f=f, s=s: oracle.loglike_batch(t, f, s, P, mag, err, 1),
                       model=lambda p, t=t: oracle.light_curve(t, p), **kw)
        croot = str(tmp_path / "cat" / ids[k])
        files = tree_files(root)
        assert files == tree_files(croot) and len(files) == 9 + 7
        for rel in files:
            assert filecmp.cmp(os.path.join(root, rel), os.path.join(croot, rel), shallow=False), (ids[k], rel)
        assert np.array_equal(res[k]["xmap"], ref["xmap"]) and res[k]["logLmap"] == ref["logLmap"]
        assert res[k]["accepted"] == ref["accepted"] and res[k]["swaps"] == ref["swaps"]


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_catalog_equals_per_target_contexts_and_oracle(hbmi, oracle):
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.catalog import Catalog
    from hb_mcmc_amd.likelihood import HBLikelihood

    real = [golden("lc_real231937440.npz"), golden("lc_real237957506.npz")]
    targets = [synth_target(n, i, oracle, gmag=(12.0 + 0.1 * i) if i % 3 == 0 else None)
               for i, n in enumerate((2, 7, 63, 64, 65, 128, 300, 1024, 2048, 1025, 1280))]
    targets += [(r["t"], r["f"], r["s"], r["mag"], r["magerr"]) for r in real]
    walkers = np.array([3, 5, 0, 64, 1, 17, 33, 128, 9, 20, 7, 40, 24], dtype=np.int32)
    P = synth.walkers(int(walkers.sum()), seed=11)
    with Catalog(targets) as cat:
        got = cat.loglike(P, walkers)
        again = cat.loglike(P, walkers)
        # a different layout on the same catalog
        w2 = walkers[::-1].copy()
        got2 = cat.loglike(P[:int(w2.sum())], w2)
    assert np.array_equal(got, again, equal_nan=True)
    o = 0
    for k, tg in enumerate(targets):
        w = int(walkers[k])
        mag = tg[3] if len(tg) > 3 else synth.MAG_DEFAULT
        err = tg[4] if len(tg) > 4 else synth.MAGERR_DEFAULT
        if w:
            # the catalog runs the one-wave kernel at every size; a lone small
            # context would take the multi-wave latency plan (other chi2 order)
            with HBLikelihood(tg[0], tg[1], tg[2], mag, err, latency_plan=False) as L:
                single = L.loglike(P[o:o + w])
            if 1024 < len(tg[0]) < 1281:
                # the catalog's pair of waves (128 lane rows) against one wave of
                # 32 cadences per lane in a lone context: other warm-chain
                # starts, chi^2 summed in another order
                assert np.array_equal(np.isnan(got[o:o + w]), np.isnan(single)), k
                ok = ~np.isnan(single)
                d = np.abs(got[o:o + w][ok] - single[ok]) / np.maximum(1.0, np.abs(single[ok]))
                assert d.max(initial=0) <= LOGL_RTOL, (k, d.max())
            else:
                assert np.array_equal(got[o:o + w], single, equal_nan=True), k
            ref = oracle.loglike_batch(tg[0], tg[1], tg[2], P[o:o + w], mag, err, 8)
            ok = ~np.isnan(ref)
            assert np.array_equal(np.isnan(got[o:o + w]), ~ok)
            rel = np.abs(got[o:o + w][ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
            assert rel.max(initial=0) <= LOGL_RTOL, (k, rel.max())
        o += w
    o = 0
    for k, tg in enumerate(targets):  # the reshuffled layout: target k owns w2[k] rows
        w = int(w2[k])
        if w:
            mag = tg[3] if len(tg) > 3 else synth.MAG_DEFAULT
            err = tg[4] if len(tg) > 4 else synth.MAGERR_DEFAULT
            with HBLikelihood(tg[0], tg[1], tg[2], mag, err) as L:
                single = L.loglike(P[o:o + w])
            if 1024 < len(tg[0]) < 1281:
                d = np.abs(got2[o:o + w] - single) / np.maximum(1.0, np.abs(single))
                assert np.array_equal(np.isnan(d), np.isnan(single)) and np.nanmax(d, initial=0) <= LOGL_RTOL, k
            else:
                assert np.array_equal(got2[o:o + w], single, equal_nan=True), k
        o += w


@pytest.mark.gpu
def test_catalog_full_deferred_queue_every_class(hbmi, oracle):
    """Times shifted by 2.5e5 days send every cadence to the reference-order
    slow path, so every wave's deferred queue fills to capacity -- in a
    catalog whose targets span the pair class (N = 1500 and 2048, the last
    region of the queue buffer, sized by each segment's launch geometry in
    hb_capi.hip catalog_layout) and the one-wave classes.  logL against the
    oracle and the same targets in per-target contexts."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.catalog import Catalog
    from hb_mcmc_amd.likelihood import HBLikelihood

    targets = []
    for i, n in enumerate((40, 300, 1024, 1100, 1500, 2048)):
        t, f, s = synth_target(n, 50 + i, oracle)
        t = t + 2.5e5
        assert (2 * np.pi * t / 10.0 ** synth.THETA_STAR[2] >= 2.0 ** 19).all()
        targets.append((t, f, s))
    walkers = np.array([9, 16, 24, 8, 40, 33], dtype=np.int32)
    P = synth.walkers(int(walkers.sum()), seed=77, roche_frac=0.1)
    with Catalog(targets) as cat:
        got = cat.loglike(P, walkers)
    o = 0
    for k, (t, f, s) in enumerate(targets):
        w = int(walkers[k])
        ref = oracle.loglike_batch(t, f, s, P[o:o + w], synth.MAG_DEFAULT, synth.MAGERR_DEFAULT, 8)
        ok = ~np.isnan(ref)
        assert np.array_equal(np.isnan(got[o:o + w]), ~ok), k
        rel = np.abs(got[o:o + w][ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
        assert rel.max(initial=0) <= LOGL_RTOL, (k, rel.max())
        with HBLikelihood(t, f, s, latency_plan=False) as L:
            single = L.loglike(P[o:o + w])
        if 1024 < len(t) < 1281:
            d = np.abs(got[o:o + w] - single) / np.maximum(1.0, np.abs(single))
            assert np.nanmax(d, initial=0) <= LOGL_RTOL, k
        else:
            assert np.array_equal(got[o:o + w], single, equal_nan=True), k
        o += w


@pytest.mark.gpu
def test_catalog_rejects_long_light_curves(hbmi, oracle):
    from hb_mcmc_amd import HBMIError
    from hb_mcmc_amd.catalog import Catalog

    with pytest.raises(HBMIError, match="2048"):
        Catalog([synth_target(64, 0, oracle), synth_target(2049, 1, oracle)])


@pytest.mark.gpu
def test_gpu_catalog_sweep_equals_single_gpu_runs(hbmi, oracle, tmp_path):
    from hb_mcmc_amd.catalog import run_catalog
    from hb_mcmc_amd.sampler import run_mcmc

    g = golden("sampler_127079833.npz")
    targets = [(g["lc_t"], g["lc_f"], g["lc_e"]), synth_target(500, 4, oracle), synth_target(1500, 5, oracle)]
    ids, periods = ["127079833", "9004", "9005"], [0.5021, 0.3157, 0.3157]
    kw = dict(niter=300, nchains=16, npast=50, run=1)
    run_catalog(targets, run_ids=ids, log10_periods=periods, out_root=str(tmp_path / "cat"), **kw)
    for k in range(3):
        root = str(tmp_path / "one" / ids[k])
        run_mcmc(*targets[k], run_id=ids[k], log10_period=periods[k], out_root=root, **kw)
        for rel in tree_files(root):
            assert filecmp.cmp(os.path.join(root, rel), os.path.join(str(tmp_path / "cat" / ids[k]), rel),
                               shallow=False), (ids[k], rel)


@pytest.mark.gpu
def test_catalog_cli_two_ranks_equals_hb_mcmc_cli(hbmi, oracle, tmp_path):
    """torchrun, 2 ranks: targets dealt by cadence count, each rank sweeps its
    own (no collective); every target's files equal the hb_mcmc CLI's."""
    import socket
    import subprocess
    import sys

    from conftest import ROOT
    from hb_mcmc_amd.hbio import write_folded_lc

    g = golden("sampler_127079833.npz")
    lcs = {"127079833": (g["lc_t"], g["lc_f"], g["lc_e"]), "9007": synth_target(640, 7, oracle)[:3],
           "9008": synth_target(1200, 8, oracle)[:3]}
    periods = {"127079833": 0.5021, "9007": 0.3157, "9008": 0.3157}
    cat_root, one_root = str(tmp_path / "cat"), str(tmp_path / "one")
    for root in [cat_root] + [os.path.join(one_root, tic) for tic in lcs]:
        d = os.path.join(root, "data", "lightcurves", "folded_lightcurves")
        os.makedirs(d, exist_ok=True)
        for tic, (t, f, e) in lcs.items():
            write_folded_lc(os.path.join(d, f"{tic}_new.txt"), t, f, e)
    pfile = str(tmp_path / "periods.txt")
    with open(pfile, "w") as fh:
        fh.writelines(f"{tic} {p}\n" for tic, p in periods.items())
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "hb_mcmc_amd.catalog",
                        "300", "--root", cat_root, "--periods", pfile, "--chains", "12", "--npast", "40"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "rank 0 target" in r.stdout and "rank 1 target" in r.stdout
    exe = os.path.join(ROOT, "hb_mcmc_amd", "lib", "hb_mcmc")
    for tic, p in periods.items():
        root = os.path.join(one_root, tic)
        r1 = subprocess.run([exe, "300", tic, str(p), "0", "--root", root, "--chains", "12", "--npast", "40",
                             "--quiet"], capture_output=True, text=True, timeout=600)
        assert r1.returncode == 0, r1.stderr
        ours = os.path.join(cat_root, tic)
        files = [rel for rel in tree_files(root) if not rel.startswith(os.path.join("data", "lightcurves", "folded"))]
        assert len(files) == 12 + 7
        for rel in files:
            assert filecmp.cmp(os.path.join(root, rel), os.path.join(ours, rel), shallow=False), (tic, rel)


# ---------------------------------------------- the reference's own targets
def test_cp_data_reader_and_folded_catalog():
    """cp_data CSV reader (hbio.read_cp_data / cp_mag_data) and the packed
    folded light curves (data/folded_catalog.npz): 111 targets, N in
    [82, 1861], every one with a cp_data row and a period; the mag block takes
    the columns dist, Gmag0, BmV0, VmG0, GmT0 (+ errors) and the reference's
    mag-file fallbacks for missing values (helpful_functions.py:377-420)."""
    from hb_mcmc_amd.hbio import DATA_DIR, cp_mag_data, load_folded_catalog, read_cp_data

    cp = read_cp_data(os.path.join(DATA_DIR, "cp_data_4-21-2022.csv"))
    assert len(cp) == 360
    r = cp["390661644"]  # first row of the CSV
    mag, err = cp_mag_data(r)
    assert np.array_equal(mag, [1063.35, 7.474916800000001, -0.1333100000000002, -0.0528777999999998,
                                -0.0545445999999998])
    assert np.array_equal(err, [0.2794518397133617, 0.24556637711065, 0.2780135623688168, 0.0595220802711405])
    mag, err = cp_mag_data(cp["440546714"])  # no Gaia: G, V-G and G-T missing
    assert mag[0] == 944.364 and (mag[1], err[0]) == (10.0, 10000.0)
    assert (mag[3], err[2]) == (0.0, 1000.0) and (mag[4], err[3]) == (0.0, 1000.0)
    assert mag[2] == -0.8790000000000013 and err[1] == 1.1352114340509436
    m0, e0 = cp_mag_data(None)
    assert np.array_equal(m0, [1000.0, 1, 1, 1, 1]) and np.array_equal(e0, np.full(4, 1e15))
    cat = load_folded_catalog()
    assert len(cat) == 111
    ns = [len(c["t"]) for c in cat]
    assert min(ns) == 82 and max(ns) == 1861
    assert all(c["tic"] in cp and c["period"] > 0 for c in cat)


def test_folded_catalog_matches_reference_files():
    """The packed arrays equal the reference's files as its reader parses
    them (mcmc_wrapper2.c:257-298 via hbio.read_folded_lc)."""
    from hb_mcmc_amd.hbio import load_folded_catalog, read_folded_lc, read_periods

    d = "/root/reference/data/lightcurves/folded_lightcurves"
    if not os.path.isdir(d):
        pytest.skip("reference tree not present (GPU box)")
    per = read_periods("/root/reference/data/lightcurves/periods.txt")
    for c in load_folded_catalog():
        t, f, e = read_folded_lc(os.path.join(d, c["name"]))
        assert np.array_equal(t, c["t"]) and np.array_equal(f, c["flux"]) and np.array_equal(e, c["sigma"])
        assert per[c["tic"]] == c["period"]


def test_mag_file_round_trip(tmp_path):
    from hb_mcmc_amd.hbio import read_mag_file, write_mag_file

    mag, err = np.array([812.5, 9.75, 0.125, -0.25, 0.0625]), np.array([0.01, 0.2, 0.3, 0.04])
    write_mag_file(str(tmp_path / "m.txt"), mag, err)
    m2, e2 = read_mag_file(str(tmp_path / "m.txt"))
    assert np.array_equal(m2, mag) and np.array_equal(e2, err)


@pytest.mark.gpu
def test_catalog_on_reference_targets_against_oracle(hbmi, oracle):
    """The 111 folded light curves with their cp_data magnitude blocks in one
    catalog (every size class N = 82..1861): logL of 8 walkers per target at
    the target's period vs the oracle (1e-10 relative; sentinel/NaN exact)."""
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.catalog import Catalog
    from hb_mcmc_amd.hbio import load_folded_catalog

    cat = load_folded_catalog()
    W = 8
    P = []
    for k, c in enumerate(cat):
        th = synth.THETA_STAR.copy()
        th[2] = np.log10(c["period"])
        th[6] = np.fmod(th[6], c["period"])
        P.append(synth.walkers(W, seed=300 + k, theta=th))
    P = np.concatenate(P)
    with Catalog([(c["t"], c["flux"], c["sigma"], c["mag"], c["magerr"]) for c in cat]) as C_:
        got = C_.loglike(P, np.full(len(cat), W, dtype=np.int32))
    for k, c in enumerate(cat):
        ref = oracle.loglike_batch(c["t"], c["flux"], c["sigma"], P[k * W:(k + 1) * W], c["mag"], c["magerr"], 8)
        g = got[k * W:(k + 1) * W]
        assert np.array_equal(np.isnan(g), np.isnan(ref)), c["name"]
        ok = ~np.isnan(ref)
        assert np.array_equal(g[ref == -5e14], ref[ref == -5e14]), c["name"]
        err = np.abs(g[ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
        assert err.max(initial=0.0) <= LOGL_RTOL, (c["name"], err.max())
