#!/bin/bash
# Focused GPU session: the given pytest node ids / -k expression ($@), one
# pytest process, stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread "$@" \
  > gpurun_out/quick.log 2>&1
rc=$?
tail -n 40 gpurun_out/quick.log | cut -c1-2000
exit $rc
