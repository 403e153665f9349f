#!/bin/bash
# experiment: slots per propose wave (kPW) variants of the device sampler
V=$PWD/hb_mcmc_amd/lib/variants
for tag in base kpw1 kpw2 kpw1t kpw2t; do
  if [ $tag = base ]; then L=$PWD/hb_mcmc_amd/lib/libhbmi.so; else L=$V/libhbmi_$tag.so; fi
  HBMI_LIB=$L timeout -k 10 120 python -u scripts/sampler_rate.py --iters 300 --device > gpurun_out/kpw_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; grep "propose blk" gpurun_out/kpw_$tag.log | head -3; tail -1 gpurun_out/kpw_$tag.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
exit 0
