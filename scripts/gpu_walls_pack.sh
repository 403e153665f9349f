#!/bin/bash
# experiment: the walls packed one coordinate per lane across the propose
# block's waves (kPW = 3 / 4 / 6 slots per block) against the shipped build.
# Variants: hb_mcmc_amd/lib/variants/libhbmi_pk<K>.so.  $1 = variant checked
# by the device-sampler GPU tests first.
V=$PWD/hb_mcmc_amd/lib/variants
T=${1:-pk6}
mkdir -p gpurun_out
HBMI_LIB=$V/libhbmi_$T.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread tests/test_dsampler.py tests/test_dsharded.py tests/test_sampler.py -m gpu \
  > gpurun_out/pk_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/pk_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for tag in base pk3 pk4 pk6; do
    if [ $tag = base ]; then L=$PWD/hb_mcmc_amd/lib/libhbmi.so; else L=$V/libhbmi_$tag.so; fi
    echo -n "$tag: "
    HBMI_LIB=$L timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null > gpurun_out/pk_rate.log
    rc=$?; tail -1 gpurun_out/pk_rate.log | cut -c1-120; [ $rc -ne 0 ] && exit $rc
  done
done
HBMI_LIB=$V/libhbmi_$T.so bash scripts/profile_dsampler.sh pk || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_pk/ds_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
