#!/bin/bash
# C5 calls: shipped library against variants (HBMI_LIB), interleaved
for r in 1 2 3; do
  for v in base $1; do
    L=""; [ $v != base ] && L="HBMI_LIB=$PWD/hb_mcmc_amd/lib/variants/libhbmi_$v.so"
    env $L timeout -k 10 120 python bench.py --config C5 --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 > gpurun_out/c5ab_tmp.log 2>&1 || exit $?
    echo "$v r=$r $(grep '^{' gpurun_out/c5ab_tmp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
