#!/bin/bash
# ds_propose timing ablations (experiment builds in lib/variants; results wrong by design)
R=$GRAFT_REPO_ROOT; V=$R/hb_mcmc_amd/lib/variants
cd /tmp && export TMPDIR=/tmp
for tag in ${TAGS:-abl1 abl2 abl3 abl4}; do
  HBMI_LIB=$V/libhbmi_$tag.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/abl_$tag -o ds -- python3 $R/scripts/sampler_rate.py --iters 100 --device > $R/gpurun_out/abl_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; grep -h "ds_propose" $R/gpurun_out/abl_$tag/ds_kernel_stats.csv | cut -d, -f1-4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
