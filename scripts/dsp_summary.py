"""Summary of scripts/gpu_dsp.sh: per run, the ranks' ms/iteration (and host
split), and from the rocprofv3 kernel traces the GPU time per kernel summed
over ranks, per rank and per timed iteration, with the swap kernels' share
(the replicated part of the sharded loop).

    python scripts/dsp_summary.py gpurun_out/dsp_TAG
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kernels(prof):
    tot = defaultdict(lambda: [0, 0.0])
    for f in glob.glob(os.path.join(prof, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "?")
                ns = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                k = tot[name]
                k[0] += 1
                k[1] += ns
    return tot


def short(name):
    name = name.replace("void ", "")
    return name.split("(")[0][:70]


def main(d):
    for js in sorted(glob.glob(os.path.join(d, "*.json"))):
        name = os.path.basename(js)[:-5]
        res = json.load(open(js))
        R, W = res["ranks"], res["W"]
        iters = res["niter"] + res["warm"]
        pr = res["per_rank"]
        ms = max(p["ms_per_iter"] for p in pr)
        print(f"== {name}: W={W} ranks={R} ({W // R} walkers a rank), tree={os.path.basename(res['tree'])}")
        print(f"   wall ms/iter (max over ranks{', gloo exchange staged through host' if R > 1 else ''}): {ms:.3f}")
        print("   host ms/iter inside step(): " + " ".join(f"{p.get('host_step_ms', float('nan')):.3f}" for p in pr))
        if "sched_build" in pr[0]:
            for k in ("sched_build", "sched_wait", "issue"):
                print(f"   host {k:12s} ms/iter: " + " ".join(f"{p[k]:.3f}" for p in pr))
        tot = kernels(os.path.join(d, "prof_" + name))
        if not tot:
            print("   (no kernel trace)")
            continue
        # per rank and iteration: all dispatches (init + warm + timed) / ranks / iterations
        gpu = sum(v[1] for v in tot.values())
        swap = sum(v[1] for k, v in tot.items() if "ds_swap" in k)
        print(f"   GPU time per rank-iteration: {gpu / R / iters / 1e3:.1f} us; swap kernels "
              f"{swap / R / iters / 1e3:.1f} us = {100.0 * swap / gpu:.1f}% of the rank's GPU time")
        for k, v in sorted(tot.items(), key=lambda kv: -kv[1][1])[:8]:
            print(f"     {short(k):70s} n={v[0]:7d} avg {v[1] / v[0] / 1e3:9.2f} us  "
                  f"{100.0 * v[1] / gpu:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1])
