#!/bin/bash
# device-sampler parity tests then its end-to-end rate and a kernel trace
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dsampler.py tests/test_glibc_math.py -m gpu -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/ds_tests.log 2>&1
rc=$?; echo "ds_tests rc=$rc"; tail -n 15 gpurun_out/ds_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/sampler_rate.py --iters 300 --device > gpurun_out/ds_rate.log 2>&1
rc=$?; echo "ds_rate rc=$rc"; tail -n 2 gpurun_out/ds_rate.log; [ $rc -ne 0 ] && exit $rc
bash scripts/profile_dsampler.sh ${1:-ds8}; rc=$?
cat gpurun_out/prof_${1:-ds8}/ds_kernel_stats.csv | cut -d, -f1-4
exit $rc
