#!/bin/bash
# GPU parity suite on the in-tree build, then the A/B session over lib/variants.
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
bash scripts/gpu_ab_session.sh ${1:-ab}
