#!/bin/bash
# C5 bench under HB_PREP_WMAX variants, interleaved
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 32 16 64; do
    HB_PREP_WMAX=$v timeout -k 10 120 python bench.py --config C5 --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 > gpurun_out/c5ab_tmp.log 2>&1 || exit $?
    echo "wmax=$v r=$r $(grep '^{' gpurun_out/c5ab_tmp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
