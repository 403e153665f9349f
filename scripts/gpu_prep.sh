#!/bin/bash
# prep-kernel change: GPU parity tests, phase clocks, bench-only kernel trace
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py tests/test_catalog.py -x -q -m gpu -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/prep_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/prep_tests.log; [ $rc -ne 0 ] && exit $rc
HBMI_LIB=$PWD/hb_mcmc_amd/lib/variants/libhbmi_ptime.so timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --sampler-iters 0 > gpurun_out/ptime.log 2>&1
rc=$?; echo "ptime rc=$rc"; grep "prep blk" gpurun_out/ptime.log | tail -4; [ $rc -ne 0 ] && exit $rc
bash scripts/profile.sh ${1:-prep}
