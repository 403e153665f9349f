#!/bin/bash
# parity of the default build, then interleaved A/B timing of lib/variants/*.so
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_catalog.py tests/test_dsampler.py -m gpu > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -n 15 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
ABLATE_STEPS=${ABLATE_STEPS:-100} timeout -k 10 600 python scripts/ablate.py --sampler-iters 0 ${AB_ARGS} > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log; exit $rc
