#!/bin/bash
# Full GPU session: parity tests, smoke, C2/C3/C5/C4 bench lines, wave clocks
# of the fused C2 launch (when the HB_WAVE_CLOCKS variant is built), bench-only
# kernel trace.  $1 = profile tag.  Stops on any fault-like exit status (>1)
# without starting further GPU work.
TAG=${1:-r01}
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-3000
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 600 python bench.py
step bench_c3 600 python bench.py --config C3 --steps 20 --warmup 3 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0
step bench_c5 600 python bench.py --config C5 --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0
step bench_c4 600 python bench.py --config C4 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0
if [ -f hb_mcmc_amd/lib/variants/libhbmi_clkf.so ]; then
  step wave_clocks 300 env HBMI_LIB=hb_mcmc_amd/lib/variants/libhbmi_clkf.so python -u scripts/wave_clocks.py --fused
fi
bash scripts/profile.sh $TAG
