#!/bin/bash
# experiment: the shipped build against a variant library
# (hb_mcmc_amd/lib/variants/libhbmi_$1.so): device-sampler GPU tests on the
# shipped build, interleaved iteration rates, one kernel trace of the shipped build
V=$PWD/hb_mcmc_amd/lib/variants
T=${1:-base}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_dsampler.py tests/test_dsharded.py tests/test_sampler.py -m gpu > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for tag in new $T; do
    if [ $tag = new ]; then L=$PWD/hb_mcmc_amd/lib/libhbmi.so; else L=$V/libhbmi_$tag.so; fi
    echo -n "$tag: "
    HBMI_LIB=$L timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null > gpurun_out/ab_rate.log
    rc=$?; tail -1 gpurun_out/ab_rate.log | cut -c1-110; [ $rc -ne 0 ] && exit $rc
  done
done
bash scripts/profile_dsampler.sh ab || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_ab/ds_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
