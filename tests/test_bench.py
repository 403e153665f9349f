"""bench.py's launch contract (CPU): `python bench.py --gpus N` starts N ranks
through torch.distributed.run by itself, and a torchrun environment whose
WORLD_SIZE disagrees with --gpus is refused.  --plumbing-check stops after the
rendezvous and one all-gather, so no GPU is needed here; the GPU bench lines
themselves are produced on the MI355X box (scripts/gpu_round.sh)."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(args, env=None, timeout=300):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def test_gpus_flag_launches_ranks():
    r = _run(["--gpus", "2", "--backend", "gloo", "--plumbing-check"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["ranks_seen"] == [0.0, 1.0]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--plumbing-check"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_config_defaults():
    sys.path.insert(0, ROOT)
    import bench

    argv = sys.argv
    try:
        for cfg, w, n in (("C2", 4096, 1024), ("C3", 4096, 20000), ("C4", 8192, 1024)):
            sys.argv = ["bench.py", "--config", cfg]
            a = bench.parse()
            assert (a.walkers, a.ncad) == (w, n), cfg
        sys.argv = ["bench.py", "--config", "C4"]
        a = bench.parse()
        assert bench.workload_label(a, 1024, 8192, 8).startswith("C4: synthetic 1024-cadence")
        assert "65536 walkers" in bench.workload_label(a, 1024, 8192, 8)
    finally:
        sys.argv = argv


def test_roofline_uses_counters_of_this_build_only(tmp_path, monkeypatch):
    """roofline(): with a PMC entry for this kernel build the bound is the fp64
    VALU (counted flops over the timed duration, VALU-issue fraction, measured
    HBM traffic) and the SURVEY 8(d) HBM figure moves to roofline.hbm; an
    entry for another build is ignored (HBM figure primary, traffic null)."""
    sys.path.insert(0, ROOT)
    import bench
    from hb_mcmc_amd._lib import kernel_build_id

    bid = kernel_build_id()
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"fp64_flop_per_call": 8.0e11, "hbm_bytes_per_call": 4.0e6, "valu_issue_cycles_per_call": 5.0e7,
             "source": "profiles/x.json"}
    (prof / "pmc_counters.json").write_text(json.dumps({bid: {"C2": entry}, "0" * 16: {"C3": entry}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    r = bench.roofline("C2", 0.04, 4096.0, 1.0e8, {"kernel_ms": 0.04})
    assert r["bound"] == "valu" and r["unit"] == "TFLOP/s"
    assert abs(r["achieved"] - 8.0e11 / 0.04e-3 / 1e12) < 1e-9
    assert abs(r["frac"] - r["achieved"] / bench.FP64_PEAK_TFLOPS) < 1e-12
    assert r["traffic"] == 4.0e6 and r["counters"]["build"] == bid
    assert abs(r["valu_issue_frac"] - 5.0e7 / (bench.SIMDS * bench.CLOCK_HZ * 0.04e-3)) < 1e-12
    assert abs(r["hbm"]["achieved"] - 1.0e8 / 0.04e-3 / 1e9) < 1e-6 and r["kernel_ms"] == 0.04
    r3 = bench.roofline("C3", 0.9, 4096.0, 2.0e9, {})
    assert r3["bound"] == "hbm" and r3["traffic"] is None and r3["counters"]["source"] is None


def test_kernel_build_id_tracks_sources():
    sys.path.insert(0, ROOT)
    from hb_mcmc_amd import _lib

    a = _lib.kernel_build_id()
    assert len(a) == 16 and a == _lib.kernel_build_id()
    for name in _lib.KERNEL_SOURCES:
        assert os.path.exists(os.path.join(_lib.CSRC, name)), name


def test_dropin_rate_takes_the_process_start_out(tmp_path):
    """bench.dropin_rate runs every leg at two lengths and reports the sampler's
    rate (niter - short) / (wall(niter) - wall(short)), the start-up and the
    wall rate beside it.  Stand-in programs here: 0.2 s of start-up plus
    0.1 ms per iteration (10 000 iterations/s), the drop-in one writing the
    HBMI_DROPIN_STATS file like libhbmi."""
    sys.path.insert(0, ROOT)
    import bench

    prog = ("#!{py}\nimport json, os, sys, time\nn = int(sys.argv[1])\ntime.sleep(0.2 + 1e-4 * n)\n"
            "p = os.environ.get('HBMI_DROPIN_STATS')\n"
            "if p:\n    json.dump({{'calls': 100 * n, 'memo_hits': 50 * n, 'batches': 6 * n, 'walkers': 50 * n,"
            " 'max_batch': 24, 'contexts_created': 1, 'profile_mode': False, 's_combine': 0.0, 's_upload': 0.0,"
            " 's_launch': 0.0, 's_download_sync': 0.0, 's_wake': 0.0, 'waiters': 40 * n}}, open(p, 'w'))\n")
    for name in ("hb_mcmc_ref_hbmi", "hb_mcmc_ref"):
        f = tmp_path / name
        f.write_text(prog.format(py=sys.executable))
        f.chmod(0o755)
    legs = (("dropin", "hb_mcmc_ref_hbmi", {}), ("reference_cpu", "hb_mcmc_ref", {}))
    out = bench.dropin_rate(1000, legs=legs, ref_dir=str(tmp_path))
    assert out["niter"] == 1000 and out["niter_short"] == 100
    for key in ("dropin", "reference_cpu"):
        leg = out[key]
        assert 7000 < leg["iters_per_s"] < 12000, leg
        assert 0.1 < leg["startup_s"] < 0.4, leg
        assert leg["iters_per_s_wall"] < 0.5 * leg["iters_per_s"], leg
    st = out["dropin"]["stats"]
    assert st["batches_per_iter"] == 6 and st["memo_hit_frac"] == 0.5 and "waiters" in st
    assert 0.5 < out["speedup_vs_reference_cpu"] < 2.0


def _settle_rank(rank, world, port, q):
    import time

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench.torch.cuda.synchronize = lambda: None  # CPU stand-in: no device here

    class A:
        backend = "gloo"

    t = torch.ones(4)

    def step(k):  # a collective per step, like the logL all-gather; rank 1 twice as slow
        time.sleep(0.0005 * (1 + rank))
        dist.all_reduce(t)

    s = bench.settle_clock(step, 30.0, None, bench.settle_agreement(A, None, world))
    dist.barrier()
    q.put((rank, s["steps"]))
    dist.destroy_process_group()


def test_settle_chunks_agree_across_ranks():
    """bench.settle_clock with world > 1: the ranks run the same number of
    settle chunks (the steps hold a collective), though one rank steps twice
    as slowly -- a time-based count per rank would leave collectives unmatched
    and hang the group (two gloo ranks on the CPU)."""
    import torch.multiprocessing as mp

    sys.path.insert(0, ROOT)
    import bench

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=_settle_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert got[0] == got[1] and got[0] % 16 == 0 and got[0] >= 16, got
