#!/bin/bash
# Interleaved device-loop iteration rate (scripts/sampler_rate.py --device) of
# the shipped build against variant libraries:
#   gpurun -- bash scripts/gpu_ds_lib_ab.sh ROUNDS "name=lib/variants/x.so ..."
ROUNDS=${1:-3}; VARS=${2:-}
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for v in new $VARS; do
    name=${v%%=*}; L=$PWD/hb_mcmc_amd/lib/libhbmi.so
    [ "$v" != "$name" ] && L=$PWD/hb_mcmc_amd/${v#*=}
    echo -n "$name $r: "
    HBMI_LIB=$L timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null > gpurun_out/ds_ab_rate.log
    rc=$?; tail -1 gpurun_out/ds_ab_rate.log | cut -c1-140; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
