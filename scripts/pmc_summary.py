"""Per-call PMC counters of one bench workload, keyed by kernel build.

    python scripts/pmc_summary.py TAG CONFIG WALKERS [NCAD]

Reads gpurun_out/pmc_TAG/*/run_counter_collection.csv (separate --pmc passes
over `bench.py`, scripts/pmc.sh), keeps the dispatches of the timed workload
(C2/C4: hb_eval_wave_kernel over 64 x WALKERS threads; C3: the eval kernel
dispatch with the largest grid (the 16-wave rows kernel); C5: the catalog's one eval launch,
hb_eval_catalog_kernel, per call = per hb_prep_kernel over all walkers) and writes

  profiles/TAG_pmc_CONFIG.json        per-call counters + derived figures
  profiles/pmc_counters.json          [build id][CONFIG] -> the same, read by bench.py

HBM bytes per call = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (MI355X_MICROARCH.md
HBM section: gfx950 tallies 128-B reads at 64 B).  Counted fp64 flops =
SQ_INSTS_VALU_FLOPS_FP64 x 64 (the counter is per wave instruction, FMA = 2).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hb_mcmc_amd._lib import kernel_build_id  # noqa: E402

tag, config, walkers = sys.argv[1], sys.argv[2], int(sys.argv[3])
ncad = int(sys.argv[4]) if len(sys.argv) > 4 else None
src = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
rows = []
for f in glob.glob(os.path.join(src, "*", "run_counter_collection.csv")):
    rows += list(csv.DictReader(open(f)))
if not rows:
    sys.exit(f"no counter files under {src}")


def is_eval(r):
    k = r["Kernel_Name"]
    if config in ("C2", "C4"):
        return "hb_eval_wave_kernel<" in k and int(r["Grid_Size"]) == 64 * walkers
    if config == "C3":  # the rows kernel (hb_eval_wave_kernel<.., WPW = 16>) or, HB_NO_ROWS=1, the block kernel
        return "hb_eval_block_kernel<" in k or "hb_eval_wave_kernel<" in k
    return "hb_eval_catalog_kernel" in k


# hb_prep_kernel: 32 / 16 walkers per 256-thread workgroup (hbk::launch_prep: the most that leave >= 256
# groups, at most 32 by default; HB_PREP_WMAX=64 for runs that allow 64)
_wmax = int(os.environ.get("HB_PREP_WMAX", "32"))
_pw = 64 if (_wmax >= 64 and walkers >= 256 * 64) else 32 if walkers >= 256 * 32 else 16
prep_grid = ((walkers + _pw - 1) // _pw) * 256
ev = collections.defaultdict(float)
calls = collections.Counter()
disp = collections.defaultdict(set)
if config == "C3":  # only the workload's (largest) block-kernel dispatches
    gmax = max(int(r["Grid_Size"]) for r in rows if is_eval(r))
for r in rows:
    c = r["Counter_Name"]
    if "hb_prep_kernel" in r["Kernel_Name"] and int(r["Grid_Size"]) == prep_grid:
        disp[c + ":prep"].add(r["Dispatch_Id"])
        continue
    if not is_eval(r) or (config == "C3" and int(r["Grid_Size"]) != gmax):
        continue
    ev[c] += float(r["Counter_Value"])
    disp[c].add(r["Dispatch_Id"])
per_call = {}
for c, tot in ev.items():
    n = len(disp[c + ":prep"]) if config == "C5" else len(disp[c])
    per_call[c] = tot / max(1, n)
d = {"tag": tag, "config": config, "walkers": walkers, "ncad": ncad, "build": kernel_build_id(),
     "per_call": per_call,
     "note": "sums over the eval dispatches of one bench step (C5: all size classes of one catalog call)"}
pc = per_call
if "FETCH_SIZE" in pc and "WRITE_SIZE" in pc:
    d["hbm_bytes_per_call"] = (2 * pc["FETCH_SIZE"] + pc["WRITE_SIZE"]) * 1024
if "SQ_INSTS_VALU_FLOPS_FP64" in pc:
    d["fp64_flop_per_call"] = pc["SQ_INSTS_VALU_FLOPS_FP64"] * 64
    d["fp64_flop_per_eval"] = d["fp64_flop_per_call"] / walkers
f64 = sum(pc.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                     "SQ_INSTS_VALU_TRANS_F64"))
if f64 and "SQ_INSTS_VALU" in pc:
    d["valu_fp64_insts_per_call"] = f64
    d["valu_other_insts_per_call"] = pc["SQ_INSTS_VALU"] - f64
    # SIMD cycles of VALU issue: fp64 at 16 lanes/clk (4 clk per wave64), the rest 2 clk
    d["valu_issue_cycles_per_call"] = 4 * f64 + 2 * (pc["SQ_INSTS_VALU"] - f64)
prof = os.path.join(ROOT, "profiles")
json.dump(d, open(os.path.join(prof, f"{tag}_pmc_{config}.json"), "w"), indent=1)
pj = os.path.join(prof, "pmc_counters.json")
allc = json.load(open(pj)) if os.path.exists(pj) else {}
allc.setdefault(d["build"], {})[config] = dict(d, source=f"profiles/{tag}_pmc_{config}.json")
json.dump(allc, open(pj, "w"), indent=1)
print(json.dumps(d, indent=1))
