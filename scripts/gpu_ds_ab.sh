#!/bin/bash
# device sampler: GPU tests, then the iteration rate under two settings of an
# experiment knob ($AB_ENV, e.g. "HB_DS_NPRIO=0"), interleaved, and one kernel trace of each
AB_ENV=${AB_ENV:-HB_DS_NO_EORD=1}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_dsampler.py tests/test_dsharded.py tests/test_sampler.py -m gpu > gpurun_out/ds_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/ds_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  echo -n "new: "; timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null | tail -1 || exit $?
  echo -n "old: "; env $AB_ENV timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null | tail -1 || exit $?
done
bash scripts/profile_dsampler.sh dse || exit $?
env $AB_ENV bash scripts/profile_dsampler.sh dsn || exit $?
for t in dse dsn; do echo $t; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_$t/ds_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
"; done
