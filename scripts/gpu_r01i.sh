#!/bin/bash
# r01i: bench-only kernel-trace profile of the current kernels, then the
# device sampler's per-phase shader clocks (HB_DS_TIMING experiment build).
mkdir -p gpurun_out
bash scripts/profile.sh r01i || exit $?
HBMI_LIB=$PWD/hb_mcmc_amd/lib/variants/libhbmi_dstiming.so timeout -k 10 200 \
  python -u scripts/sampler_rate.py --iters 150 --device > gpurun_out/ds_timing.log 2>&1
rc=$?; echo "ds_timing rc=$rc"; grep -c "propose blk" gpurun_out/ds_timing.log; tail -3 gpurun_out/ds_timing.log
exit $rc
