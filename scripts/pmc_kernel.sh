#!/bin/bash
# One rocprofv3 PMC pass (kernel trace only) over the C2 likelihood bench (or
# BENCH_ARGS), summarised per kernel: dispatches, waves and each counter per
# dispatch and per wave.  $1 = tag, $2 = counter list (one pass: at most 8 SQ_).
TAG=${1:-k}
SET=$2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmck_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES $SET --output-format csv -d $OUT/run -o run \
  -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 --kernel-samples 5 ${BENCH_ARGS} > $OUT/run.log 2>&1
rc=$?; echo "pmc [$SET] rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/run.log; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = sorted(glob.glob(out + "/run/**/*counter_collection.csv", recursive=True))
rows = list(csv.DictReader(open(f[0])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in agg.items():
    n = len(disp[k]); w = c["SQ_WAVES"] or 1
    print(f"{k}  dispatches {n}  waves/dispatch {w/n:.0f}")
    for name, v in sorted(c.items()):
        print(f"    {name:28s} per dispatch {v/n:14.1f}   per wave {v/w:10.2f}")
PY
