#!/bin/bash
# rocprof kernel stats of the C5 bench with and without the pair plan
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in pair nopair; do
  mkdir -p $R/gpurun_out/pairprof_$v
  if [ $v = nopair ]; then export HB_NO_PAIR=1; else unset HB_NO_PAIR; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pairprof_$v -o c5 \
    -- python3 $R/bench.py --config C5 --steps 50 --warmup 5 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 \
    > $R/gpurun_out/pairprof_$v/stdout.log 2>&1 || exit 1
done
