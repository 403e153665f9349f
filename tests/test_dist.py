"""Multi-rank PT-MCMC (hb_mcmc_amd/dist.py): temperature slots sharded over
ranks, logL all-gathered, tempering swaps replayed on every rank, records of
boundary-crossing chains exchanged all-to-all.  gloo on CPU, world_size 2
and 3; each rank's likelihood is the oracle (standing in for its GPU).

The sharded run must reproduce the REFERENCE's own trace byte for byte
(tests/golden/sampler_127079833.npz, the same fixture as test_sampler.py) and,
for uneven shards / other ladders, the single-process sampler's files.
"""
import filecmp
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import golden

import _dist_worker


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(world, case, out_root, result_path):
    mp.spawn(_dist_worker.worker, args=(world, free_port(), case, out_root, result_path), nprocs=world, join=True)
    return np.load(result_path)


def tree_files(root):
    out = []
    for d, _, fs in os.walk(root):
        out += [os.path.relpath(os.path.join(d, f), root) for f in fs]
    return sorted(out)


def test_shard_bounds():
    from hb_mcmc_amd.dist import shard

    for W in (4, 7, 50, 4096, 65536):
        for R in (1, 2, 3, 8):
            b = [shard(W, r, R) for r in range(R)]
            assert b[0][0] == 0 and b[-1][1] == W
            assert all(b[i][1] == b[i + 1][0] for i in range(R - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


@pytest.mark.slow
def test_two_ranks_match_reference_trace(tmp_path):
    g = golden("sampler_127079833.npz")
    case = dict(t=g["lc_t"], f=g["lc_f"], e=g["lc_e"], niter=int(g["niter"][0]), run_id="127079833",
                log10_period=0.5021, nchains=50)
    res = spawn(2, case, str(tmp_path), str(tmp_path / "res.npz"))
    for i, name in enumerate(g["file_names"]):
        with open(os.path.join(str(tmp_path), str(name)), "rb") as fh:
            assert fh.read() == bytes(g[f"file{i}"]), name
    suf = "127079833_gmag_OMP_0"
    with open(os.path.join(str(tmp_path), f"data/chains/chain.{suf}.dat"), "rb") as fh:
        assert fh.read() == bytes(g["chain_txt"])
    with open(os.path.join(str(tmp_path), f"data/logL/logL.{suf}.dat"), "rb") as fh:
        assert fh.read() == bytes(g["logl_txt"])
    assert int(res["evals"]) == 1 + 50 + 1200 * 50
    assert int(res["moved"]) > 0  # chains did cross the rank boundary


@pytest.mark.parametrize("world,W,ladder", [(2, 7, 0), (3, 11, 0), (3, 120, 1)])
def test_uneven_shards_match_single_process(tmp_path, oracle, world, W, ladder):
    from hb_mcmc_amd.sampler import run_mcmc

    g = golden("sampler_127079833.npz")
    t, f, e = g["lc_t"][:400], g["lc_f"][:400], g["lc_e"][:400]
    case = dict(t=t, f=f, e=e, niter=260, run_id="42", log10_period=0.5021, nchains=W, npast=20, ladder=ladder,
                run=3)
    dist_root, single_root = tmp_path / "dist", tmp_path / "single"
    res = spawn(world, case, str(dist_root), str(tmp_path / "res.npz"))
    mag, err = np.array([1000.0, 1, 1, 1, 1]), np.full(4, 1e15)
    ref = run_mcmc(t, f, e, niter=260, run_id="42", log10_period=0.5021, run=3, nchains=W, npast=20,
                   ladder=ladder, out_root=str(single_root), nthreads=2,
                   loglik=lambda P: oracle.loglike_batch(t, f, e, P, mag, err, 1),
                   model=lambda p: oracle.light_curve(t, p))
    files = tree_files(str(single_root))
    assert files == tree_files(str(dist_root)) and len(files) == W + 7
    for rel in files:
        assert filecmp.cmp(os.path.join(str(single_root), rel), os.path.join(str(dist_root), rel), shallow=False), rel
    assert np.array_equal(res["xmap"], ref["xmap"]) and float(res["logLmap"]) == ref["logLmap"]
    assert int(res["accepted"]) == ref["accepted"] and int(res["swaps"]) == ref["swaps"]
    assert int(res["evals"]) == ref["loglik_evals"]
    assert int(res["moved"]) > 0


def run_dist_cli(tmp, nproc, backend):
    import subprocess
    import sys

    from conftest import ROOT
    from test_sampler import stage_input

    g = stage_input(tmp)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m", "hb_mcmc_amd.dist",
                        "1200", "127079833", "0.5021", "0", "--root", tmp, "--backend", backend],
                       capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return g, r.stdout


@pytest.mark.gpu
def test_dist_cli_rccl_one_rank_gpu(tmp_path):
    """torchrun + RCCL (nccl backend), the GPU likelihood: matches the reference trace."""
    from test_sampler import assert_gpu_run_matches_reference

    g, out = run_dist_cli(str(tmp_path), 1, "nccl")
    assert "done: 1200 iterations on 1 ranks" in out
    assert_gpu_run_matches_reference(tmp_path, g)


@pytest.mark.gpu
def test_dist_cli_two_ranks_gpu_likelihood(tmp_path):
    """Two ranks (gloo between them, both evaluating on the box's one GPU)."""
    from test_sampler import assert_gpu_run_matches_reference

    g, out = run_dist_cli(str(tmp_path), 2, "gloo")
    assert "done: 1200 iterations on 2 ranks" in out
    assert_gpu_run_matches_reference(tmp_path, g)
