#!/bin/bash
mkdir -p gpurun_out
ABLATE_STEPS=100 timeout -k 10 600 python scripts/ablate.py --sampler-iters 0 --dropin-iters 0 > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log; [ $rc -ne 0 ] && exit $rc
bash scripts/pmc.sh x1 "SQ_INSTS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64"
