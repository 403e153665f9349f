#!/bin/bash
# parity of the default build (likelihood, catalog, device sampler), then the
# wave-clock readout of the clock variants and the interleaved A/B timing
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_catalog.py tests/test_dsampler.py -m gpu > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -n 6 gpurun_out/ab_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_exp.sh
