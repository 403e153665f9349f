"""The N > 1 bench path the driver's scaling run executes (`bench.py --gpus N`),
rehearsed end to end on the GPU box: two ranks launched by bench.py itself
(torch.distributed.run child), backend gloo so both ranks can share the box's
one GPU, the timed likelihood steps with the overlapped logL all-gather
(mcmc_wrapper2.c:554-563 needs every walker's logL), then the sharded
device-resident sampler (`sampler_e2e_sharded`: one all-gather of logL + edge
records per iteration).  Small step counts; the line must
show what the process group saw."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(args, timeout=240):
    e = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                       text=True, timeout=timeout, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 only
    return json.loads(lines[0])


SMALL = ["--gpus", "2", "--backend", "gloo", "--steps", "5", "--warmup", "2", "--kernel-samples", "3",
         "--sampler-iters", "4", "--no-cpu-baseline", "--dropin-iters", "0", "--prior-steps", "0"]


@pytest.mark.parametrize("config,w", [("C2", 4096), ("C4", 8192)])
def test_bench_two_ranks_end_to_end(config, w):
    line = _bench(SMALL + ["--config", config])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["steps"] == 5
    assert line["config"]["walkers_per_gpu"] == w and line["config"]["global_walkers"] == 2 * w
    pg = line["process_group"]
    assert pg["world_size"] == 2 and pg["backend"] == "gloo" and pg["ranks_seen"] == [0, 1]
    assert [r["local_rank"] for r in pg["ranks"]] == [0, 1]
    assert line["allgather_check"]["ok"] is True and line["allgather_check"]["doubles_per_step"] == 2 * w
    e2e = line["sampler_end_to_end"]
    assert e2e["ranks"] == 2 and e2e["walkers"] == 2 * w and e2e["walkers_per_rank"] == w
    ds = e2e["device_loop_sharded"]
    assert ds["ms_per_iter"] > 0 and ds["exchange_bytes_per_rank_per_iter"] > 0
    assert line["nonfinite_logl_last_batch"] <= w // 100


def test_bench_two_ranks_catalog():
    line = _bench(SMALL + ["--config", "C5", "--targets", "24", "--walkers-per-target", "16"])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["config"]["global_walkers"] == 24 * 16
    assert line["process_group"]["ranks_seen"] == [0, 1]
