#!/bin/bash
# rocprofv3 kernel-trace summary of the device-resident sampler loop.  $1 = tag
TAG=${1:-ds}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o ds \
  -- python3 $R/scripts/sampler_rate.py --iters 200 --device ${DS_ARGS} > $R/gpurun_out/prof_$TAG/stdout.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $R/gpurun_out/prof_$TAG/stdout.log
exit $rc
