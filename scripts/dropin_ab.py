"""Interleaved A/B of the drop-in's policy knobs (hb_capi.hip DropPolicy,
hb_dropin.hpp): the reference sampler relinked against libhbmi.so
(bench.dropin_rate) under several HBMI_DROPIN_* environments, `rounds`
rounds in turn, so box drift hits every variant alike.

    python scripts/dropin_ab.py [niter] [rounds] > gpurun_out/rNN_dropin_ab.txt
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

VARIANTS = {
    "base": {},
    "memo_off": {"HBMI_DROPIN_MEMO": "0"},
    "block": {"HBMI_DROPIN_BLOCK": "1"},
    "spin_win": {"HBMI_DROPIN_SPIN_US": "300", "HBMI_DROPIN_WINDOW_US": "30"},
    "block_win": {"HBMI_DROPIN_BLOCK": "1", "HBMI_DROPIN_WINDOW_US": "30"},
    "lanes2_block": {"HBMI_DROPIN_LANES": "2", "HBMI_DROPIN_BLOCK": "1"},
    "omp_passive": {"OMP_WAIT_POLICY": "passive"},
    "block_omp_passive": {"HBMI_DROPIN_BLOCK": "1", "OMP_WAIT_POLICY": "passive"},
    "chain1": {"HBMI_DROPIN_CHAIN": "1"},
    "chain2": {"HBMI_DROPIN_CHAIN": "2"},
    "chain4": {"HBMI_DROPIN_CHAIN": "4"},
    "chain8": {"HBMI_DROPIN_CHAIN": "8"},
    "chain64": {"HBMI_DROPIN_CHAIN": "64"},
    "chain4_omp_passive": {"HBMI_DROPIN_CHAIN": "4", "OMP_WAIT_POLICY": "passive"},
}


def main():
    niter = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    only = sys.argv[3].split(",") if len(sys.argv) > 3 else list(VARIANTS)
    res = {k: [] for k in only}
    for r in range(rounds):
        for k in only:
            out = bench.dropin_rate(niter, legs=((k, "hb_mcmc_ref_hbmi", VARIANTS[k]),))
            leg = out.get(k, {})
            res[k].append(leg.get("iters_per_s"))
            st = leg.get("stats", {})
            print(json.dumps({"round": r, "variant": k, "iters_per_s": leg.get("iters_per_s"),
                              "error": leg.get("error"),
                              "batches_per_iter": st.get("batches_per_iter"), "mean_batch": st.get("mean_batch"),
                              "us_per_batch": st.get("us_per_batch"),
                              "us_wake_per_waiter": st.get("us_wake_per_waiter")}), flush=True)
    for env in ({}, {"OMP_WAIT_POLICY": "passive"}):
        ref = bench.dropin_rate(niter, legs=(("reference_cpu", "hb_mcmc_ref", env),)).get("reference_cpu", {})
        print(json.dumps({"reference_cpu_iters_per_s": ref.get("iters_per_s"), "env": env}))
    for k, v in res.items():
        ok = sorted(x for x in v if x)
        print(f"{k:18s} median {ok[len(ok) // 2] if ok else float('nan'):9.1f} it/s  runs {[round(x or 0) for x in v]}")


if __name__ == "__main__":
    main()
