#!/bin/bash
# A/B session (scripts/gpu_ab_session.sh) plus per-variant PMC passes of the
# eval kernel: instruction counts, LDS conflicts and waits, I/K-cache hits.
bash scripts/gpu_ab_session.sh ab3 || exit 1
for v in a_base_stride d_gq_sel3_odd; do
  L=$GRAFT_REPO_ROOT/hb_mcmc_amd/lib/variants/libhbmi_$v.so
  HBMI_LIB=$L bash scripts/pmc_kernel.sh pmc_$v "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" > gpurun_out/ab3/pmc_$v.log 2>&1 || exit 1
  HBMI_LIB=$L bash scripts/pmc_kernel.sh icache_$v "SQC_ICACHE_HITS SQC_ICACHE_MISSES" > gpurun_out/ab3/icache_$v.log 2>&1 || exit 1
  HBMI_LIB=$L bash scripts/pmc_kernel.sh dcache_$v "SQC_DCACHE_HITS SQC_DCACHE_MISSES" > gpurun_out/ab3/dcache_$v.log 2>&1 || exit 1
done
