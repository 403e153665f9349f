#!/bin/bash
# device sampler: GPU tests + iteration rate (W = 4096, N = 1024) + kernel trace
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_dsampler.py tests/test_dsharded.py tests/test_sampler.py -m gpu > gpurun_out/ds_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/ds_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null | tail -1 || exit $?; done
bash scripts/profile_dsampler.sh dsq || exit $?
HB_DS_SPLIT_ACCEPT=1 bash scripts/profile_dsampler.sh dsq2 || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_dsq/ds_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
[ -f gpurun_out/prof_dsq2/ds_kernel_stats.csv ] && python3 -c "
import csv
print('split accept:')
for r in csv.DictReader(open('gpurun_out/prof_dsq2/ds_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
