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
