"""Drop-in leg probes (GPU box): the fixed per-process cost inside the leg's
wall time, and a rocprofv3 kernel trace of the relinked reference sampler.

  python scripts/dropin_prof.py fixed [niters...]   one JSON line per run
  python scripts/dropin_prof.py prof OUTDIR [niter]  rocprofv3 --kernel-trace --stats

The sampler is oracle/_ref/hb_mcmc_ref_hbmi (mcmc_wrapper2.c relinked against
libhbmi.so, bench.dropin_rate); this process never touches HIP, the profiler
runs the sampler binary directly after `--`.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

EXE = os.path.join(ROOT, "oracle", "_ref", "hb_mcmc_ref_hbmi")


def run(niter, prefix=(), extra=None):
    g = np.load(os.path.join(ROOT, "tests", "golden", "sampler_127079833.npz"))
    with tempfile.TemporaryDirectory() as tmp:
        bench.dropin_workdir(tmp, g)
        stats = os.path.join(tmp, "stats.json")
        env = dict(os.environ, HBREF_ROOT=tmp, HBMI_DROPIN_STATS=stats, **(extra or {}))
        t0 = time.perf_counter()
        r = subprocess.run(list(prefix) + [EXE, str(niter), "127079833", "0.5021", "0"], cwd=tmp,
                           capture_output=True, text=True, timeout=900, env=env)
        dt = time.perf_counter() - t0
        st = json.load(open(stats)) if os.path.exists(stats) else None
    return {"niter": niter, "rc": r.returncode, "wall_s": dt, "iters_per_s": niter / dt, "stats": st,
            "stderr": r.stderr[-300:] if r.returncode else ""}


def main():
    mode = sys.argv[1]
    if mode == "fixed":
        ns = [int(x) for x in sys.argv[2:]] or [50, 1000, 3000]
        rows = []
        for n in ns:
            rows.append(run(n))
            print(json.dumps({k: v for k, v in rows[-1].items() if k != "stats"}), flush=True)
        x = np.array([r["niter"] for r in rows], float)
        y = np.array([r["wall_s"] for r in rows])
        a, b = np.polyfit(x, y, 1)
        print(json.dumps({"fit": {"s_per_iter": a, "fixed_s": b, "steady_iters_per_s": 1 / a}}), flush=True)
    elif mode == "prof":
        out = os.path.abspath(sys.argv[2])
        n = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
        os.makedirs(out, exist_ok=True)
        r = run(n, prefix=["rocprofv3", "--kernel-trace", "--stats", "-d", out, "-o", "run", "--"])
        print(json.dumps(r), flush=True)
        sys.exit(r["rc"])


if __name__ == "__main__":
    main()
