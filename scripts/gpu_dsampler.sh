#!/bin/bash
# Device-sampler GPU session: glibc-exact device math, device vs host sampler
# state, reference trace, then the end-to-end iteration rate.  Stops on any
# fault-like exit status (>1) without starting further GPU work.
mkdir -p gpurun_out
FAILED=0
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  [ $rc -ne 0 ] && FAILED=1
  return 0
}
step ds_tests 400 python -u -m pytest tests/test_glibc_math.py tests/test_dsampler.py -m gpu -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread
step ds_rate 200 python -u scripts/sampler_rate.py --iters 300 --device
step host_rate 200 python -u scripts/sampler_rate.py --iters 300
exit $FAILED
