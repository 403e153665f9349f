#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py for each lib/variants/*.so
# (per-instantiation kernel durations); BENCH_ARGS selects the workload.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for l in $R/hb_mcmc_amd/lib/variants/libhbmi_*.so; do
  tag=$(basename $l .so); out=$R/gpurun_out/pv_$tag
  mkdir -p $out
  HBMI_LIB=$l timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run \
    -- python3 $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline --sampler-iters 0 ${BENCH_ARGS} > $out/stdout.log 2>&1 || exit $?
  echo "== $tag"; python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
done
