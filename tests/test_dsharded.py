"""Sharded device-resident PT-MCMC (ShardedDeviceSampler,
hb_dsampler_create_shard / step_begin / step_end): each rank proposes,
evaluates and tests its own slots on its GPU; one all-gather per iteration
carries logL by slot plus the records of the chains near each shard's edges
(mcmc_wrapper2.c:554-563).

CPU: the edge-window rule the exchange relies on -- with nlv dependency levels
a chain moves at most nlv slots, so every chain that leaves a shard starts in
the min(nlv, smallest shard) slots at one of its edges -- checked on random
schedules and accept patterns, including shards smaller than nlv.

GPU (ranks share the box's one GPU over gloo): the sharded run equals the
single-process device sampler bit for bit -- every slot's state, logL, chain
id, RNG stream and history, the counters and the MAP point -- at W = 65 536
(BASELINE config C4's ensemble, 50-rung ladder repeated) and on uneven shards;
the CLI (`python -m hb_mcmc_amd.dist --device-sampler`) reproduces the
reference's own 1200-iteration trace on 2 ranks.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from test_dsampler import levels


def _edge_rule(W, R, rng):
    from hb_mcmc_amd.dist import shard

    b = rng.integers(0, W, W)
    lv = levels(b, W)
    nlv = int(lv.max(initial=0))
    idx = np.arange(W)
    for level in range(1, nlv + 1):
        for x in b[lv == level]:
            if rng.random() < 0.7:  # accepted swap
                idx[x], idx[x + 1] = idx[x + 1], idx[x]
    bounds = [shard(W, r, R) for r in range(R)]
    nlmin = min(hi - lo for lo, hi in bounds)
    ke = min(nlv, nlmin)
    pos = np.empty(W, dtype=np.int64)
    pos[idx] = np.arange(W)  # new slot of each chain (chain c started in slot c)
    for lo, hi in bounds:
        window = set(range(lo, min(hi, lo + ke))) | set(range(max(lo, hi - ke), hi))
        for c in range(lo, hi):
            if not (lo <= pos[c] < hi):
                assert c in window, (W, R, lo, hi, c, pos[c], nlv)
        assert abs(pos - np.arange(W)).max() <= nlv


@pytest.mark.parametrize("W,R", [(7, 3), (50, 3), (100, 8), (4096, 2), (65536, 8)])
def test_edge_windows_cover_every_leaving_chain(W, R):
    rng = np.random.default_rng(W + R)
    for _ in range(3):
        _edge_rule(W, R, rng)


def test_sharded_symbols_exported():
    from hb_mcmc_amd import _lib, sampler

    lib = sampler._declare(_lib.lib())
    for name in ("hb_dsampler_create_shard", "hb_dsampler_step_begin", "hb_dsampler_step_end",
                 "hb_dsampler_exchange_cap", "hb_dsampler_stream", "hb_dsampler_host_times"):
        assert hasattr(lib, name)


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sharded(tmp, W, niter, ladder, npast, n, ranks, backend="gloo", exchange=False):
    out = os.path.join(str(tmp), f"sharded_{W}_{ranks}.npz")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "tests", "_dsharded_worker.py"), out, str(W), str(niter), str(ladder),
                        str(npast), str(n), backend] + (["x"] if exchange else []),
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return np.load(out)


def _single(W, niter, ladder, npast, n):
    from hb_mcmc_amd import synth
    from hb_mcmc_amd.dsampler import DeviceSampler
    from hb_mcmc_amd.likelihood import HBLikelihood
    from hb_mcmc_amd.sampler import SlotSampler

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _dsharded_worker as wk

    t, f, s = wk.dataset(n, synth, HBLikelihood, 0)
    with HBLikelihood(t, f, s) as L:
        S = SlotSampler(niter, W, synth.THETA_STAR[2], 0, W, run=0, npast=npast, ladder=ladder)
        with DeviceSampler(S, L) as D:
            D.init_logl()
            for it in range(niter):
                D.step(it)
            x, ll, xmap, lmap, _ = D.gather()
            D.download()
        _, _, cid = S.get()
        arrs = S.state_arrays()
        st = S.stats()
        S.close()
    return dict(x=x, logl=ll, cid=cid, xmap=xmap, logLmap=lmap, seeds=arrs["seeds"],
                hist=arrs["history"].reshape(W, -1), st=st)


def _compare(a, b):
    assert np.array_equal(a["cid"], b["cid"]), "chain ids by slot"
    assert np.array_equal(a["x"], b["x"]), "states"
    assert np.array_equal(a["logl"], b["logl"], equal_nan=True), "logL"
    assert np.array_equal(a["seeds"].astype(np.int64), b["seeds"]), "RNG streams"
    assert np.array_equal(a["hist"], b["hist"]), "history"
    assert np.array_equal(a["xmap"], b["xmap"]) and float(a["logLmap"]) == b["logLmap"], "MAP"
    st = b["st"]
    assert list(a["sums"].astype(np.int64)) == [st["acc"], st["DEacc"], st["DEtrial"], st["cold_acc"], st["nswap"]]
    assert int(a["atrial"]) == st["atrial"]
    assert st["nswap"] > 0


@pytest.mark.gpu
def test_sharded_device_sampler_c4_equals_single_process(tmp_path):
    """W = 65 536 (C4's ensemble), N = 1024, 2 ranks: bit-identical to one process."""
    W, niter, ladder, npast, n = 65536, 30, 1, 20, 1024
    a = _sharded(tmp_path, W, niter, ladder, npast, n, 2)
    b = _single(W, niter, ladder, npast, n)
    _compare(a, b)
    # the exchange stays small: logL of a shard plus a few dozen edge records
    assert float(a["exchanged"]) / niter < W / 2 + 2 * 64 * 24


@pytest.mark.gpu
def test_rccl_exchange_one_rank_equals_device_sampler(tmp_path):
    """The RCCL branch of ShardedDeviceSampler.step on one GPU: world size 1
    under backend nccl with the exchange forced, so every iteration runs
    ds_pack -> all_gather_into_tensor on the sampler's stream -> ds_swap's
    import (the C4 exchange, mcmc_wrapper2.c:554-563).  W = 4096, 100
    iterations: bit-identical to the plain DeviceSampler."""
    W, niter, ladder, npast, n = 4096, 100, 1, 20, 1024
    a = _sharded(tmp_path, W, niter, ladder, npast, n, 1, backend="nccl", exchange=True)
    b = _single(W, niter, ladder, npast, n)
    _compare(a, b)
    assert float(a["exchanged"]) >= niter * W  # the logL block went through RCCL every iteration


@pytest.mark.gpu
@pytest.mark.parametrize("W,ranks,ladder", [(50, 3, 0), (7, 3, 0), (6000, 4, 1)])
def test_sharded_device_sampler_uneven_shards(tmp_path, W, ranks, ladder):
    """Uneven shards, shards smaller than the level count (W = 7 over 3 ranks),
    the LDS swap path (W <= 4266) and the global one (W = 6000)."""
    niter, npast, n = 40, 20, 256
    a = _sharded(tmp_path, W, niter, ladder, npast, n, ranks)
    b = _single(W, niter, ladder, npast, n)
    _compare(a, b)


@pytest.mark.gpu
def test_sharded_device_cli_reproduces_reference_trace(tmp_path):
    """`python -m hb_mcmc_amd.dist --device-sampler` on 2 ranks: the reference's
    own `HB_MCMC 1200 127079833 0.5021 0` output files."""
    from test_sampler import assert_gpu_run_matches_reference, stage_input

    g = stage_input(str(tmp_path))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "hb_mcmc_amd.dist",
                        "1200", "127079833", "0.5021", "0", "--root", str(tmp_path), "--backend", "gloo",
                        "--device-sampler"],
                       capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "done: 1200 iterations on 2 ranks" in r.stdout
    assert_gpu_run_matches_reference(tmp_path, g)
