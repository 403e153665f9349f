#!/bin/bash
# parity of the default build (likelihood + catalog + device sampler), then
# interleaved A/B of lib/variants/*.so on C2, C5 and the device-resident loop
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_catalog.py tests/test_dsampler.py -m gpu > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/ab_pytest.log; [ $rc -gt 1 ] && exit $rc
ABLATE_STEPS=100 timeout -k 10 300 python scripts/ablate.py --sampler-iters 0 --config C5 > gpurun_out/ab_c5.log 2>&1 || exit $?
ABLATE_STEPS=200 timeout -k 10 200 python scripts/ablate.py --sampler-iters 0 > gpurun_out/ab_c2.log 2>&1 || exit $?
ABLATE_MODE=sampler ABLATE_STEPS=200 timeout -k 10 300 python scripts/ablate.py > gpurun_out/ab_ds.log 2>&1 || exit $?
cat gpurun_out/ab_c5.log gpurun_out/ab_c2.log gpurun_out/ab_ds.log
