#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py (no PMC here).  $1 = tag
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench \
  -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 ${BENCH_ARGS} > $R/gpurun_out/prof_$TAG/bench_stdout.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $R/gpurun_out/prof_$TAG/bench_stdout.log
find $R/gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
