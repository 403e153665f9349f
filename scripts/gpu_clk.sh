#!/bin/bash
# per-phase wave clocks of two eval-kernel builds (HB_WAVE_CLOCKS variants)
O=gpurun_out/clk; mkdir -p $O
for v in clk2 clk3; do
  HBMI_LIB=$GRAFT_REPO_ROOT/hb_mcmc_amd/lib/variants/libhbmi_$v.so timeout -k 10 120 python3 scripts/wave_clocks.py > $O/$v.json 2>$O/$v.err || { tail -3 $O/$v.err; exit 1; }
done
