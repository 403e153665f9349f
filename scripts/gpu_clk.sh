#!/bin/bash
# per-phase wave clocks of the HB_WAVE_CLOCKS variants in lib/variants
# (libhbmi_clk*.so)
O=gpurun_out/clk; mkdir -p $O
for l in $GRAFT_REPO_ROOT/hb_mcmc_amd/lib/variants/libhbmi_clk*.so; do
  v=$(basename $l .so)
  HBMI_LIB=$l timeout -k 10 120 python3 scripts/wave_clocks.py > $O/$v.json 2>$O/$v.err || { tail -3 $O/$v.err; exit 1; }
done
