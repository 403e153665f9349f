#!/bin/bash
# One rocprofv3 PMC pass (kernel trace only, 6 SQ counters) over the
# device-resident PT-MCMC loop (sampler_rate.py --device, W = 4096, N = 1024):
# per-kernel wave cycles, VALU / SALU / LDS instructions, VALU-active and
# wait cycles of ds_propose, ds_swap, the prep and the eval + Hastings kernels.
TAG=${1:-ds}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
  --output-format csv -d $OUT/run -o run -- python3 $R/scripts/sampler_rate.py --device --iters 60 > $OUT/run.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = sorted(glob.glob(out + "/run/**/*counter_collection.csv", recursive=True))
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
print(f"{'kernel':40s} {'disp':>5s} {'waves':>8s} {'VALU/wave':>10s} {'SALU/wave':>10s} {'VALUact/wcyc':>12s} {'wait/wcyc':>10s}")
for k, c in agg.items():
    n = len(disp[k]); w = c["SQ_WAVES"] or 1; wc = c["SQ_WAVE_CYCLES"] or 1
    print(f"{k:40s} {n:5d} {w/n:8.0f} {c['SQ_INSTS_VALU']/w:10.0f} {c['SQ_INSTS_SALU']/w:10.0f} "
          f"{c['SQ_ACTIVE_INST_VALU']/wc:12.3f} {c['SQ_WAIT_INST_ANY']/wc:10.3f}")
PY
