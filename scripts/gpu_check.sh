#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Stops on any fault-like
# exit status (>1: abort/segv/timeout) without starting further GPU work.
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 100 --warmup 10 ${BENCH_ARGS}
