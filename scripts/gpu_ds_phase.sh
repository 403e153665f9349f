#!/bin/bash
# ds_propose phase clocks (HB_DS_TIMING variant builds in lib/variants) and
# kernel times of the timing build and two ablations (results wrong by design)
R=$GRAFT_REPO_ROOT; V=$R/hb_mcmc_amd/lib/variants
mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
for tag in ${TAGS:-dstime dsabl1 dsabl2}; do
  HBMI_LIB=$V/libhbmi_$tag.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/ph_$tag -o ds -- python3 $R/scripts/sampler_rate.py --iters 150 --device > $R/gpurun_out/ph_$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; grep -E "slot|swap:" $R/gpurun_out/ph_$tag.log; grep -h "ds_propose" $R/gpurun_out/ph_$tag/ds_kernel_stats.csv | cut -d, -f1-4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
