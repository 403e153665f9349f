#!/bin/bash
# rocprofv3 PMC passes (kernel-trace only, no sys/runtime trace) over a short bench.
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for set in "$@"; do
  [ $i -eq 0 ] && { i=1; continue; }   # first arg is the tag
  name=$(echo $set | tr ' ' '_' | cut -c1-60)
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/$name -o run \
     -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 --prior-steps 0 --settle-ms 0 --two-stream-steps 0 ${BENCH_ARGS} > $OUT/$name.log 2>&1
  rc=$?; echo "pmc [$set] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit $rc; fi
done
