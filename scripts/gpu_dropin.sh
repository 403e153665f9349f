#!/bin/bash
# drop-in path: the relinked reference sampler's trace test, the C-ABI GPU tests, and its rate
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_sampler.py tests/test_capi.py -m gpu > gpurun_out/dropin_pytest.log 2>&1
rc=$?; tail -n 4 gpurun_out/dropin_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "
import json, bench
print(json.dumps(bench.dropin_rate(200), indent=1))
"
