"""Rank body of tests/test_dist.py (spawned with torch.multiprocessing).

Test infrastructure: the likelihood provider here is the oracle (a CPU
restatement of likelihood3.c), standing in for each rank's GPU so that the
sharded sampler's bookkeeping can be checked on CPU with gloo."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def worker(rank, world, port, case, out_root, result_path):
    import numpy as np
    import torch.distributed as dist

    from hb_mcmc_amd.dist import run_sharded
    from oracle import Oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = Oracle()
        t, f, e = case["t"], case["f"], case["e"]
        mag = np.array([1000.0, 1, 1, 1, 1])
        err = np.full(4, 1e15)
        res = run_sharded(t, f, e, niter=case["niter"], run_id=case["run_id"], log10_period=case["log10_period"],
                          run=case.get("run", 0), nchains=case["nchains"], npast=case.get("npast", 500),
                          ladder=case.get("ladder", 0), nthreads=2, out_root=out_root if rank == 0 else out_root,
                          loglik=lambda P: orc.loglike_batch(t, f, e, P, mag, err, 1),
                          model=lambda p: orc.light_curve(t, p))
        if rank == 0:
            np.savez(result_path, xmap=res["xmap"], logLmap=res["logLmap"], accepted=res["accepted"],
                     swaps=res["swaps"], evals=res["loglik_evals"], moved=res["records_moved"])
    finally:
        dist.destroy_process_group()
