#!/bin/bash
# Experiment session: wave-clock readout of the clock variants, then the
# interleaved A/B timing of every lib/variants/*.so on the C2 bench.
mkdir -p gpurun_out
V=hb_mcmc_amd/lib/variants
for c in $V/libhbmi_*clk*.so; do
  [ -e "$c" ] || continue
  echo "== $c"
  HBMI_LIB=$c timeout -k 10 120 python scripts/wave_clocks.py ${CLK_ARGS} > gpurun_out/clk_$(basename $c .so).json 2>&1
  rc=$?; cat gpurun_out/clk_$(basename $c .so).json | tail -30; [ $rc -ne 0 ] && exit $rc
done
ABLATE_STEPS=${ABLATE_STEPS:-100} timeout -k 10 600 python scripts/ablate.py --sampler-iters 0 --dropin-iters 0 ${AB_ARGS} > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log; exit $rc
