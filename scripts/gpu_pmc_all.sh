#!/bin/bash
# PMC passes (kernel trace only, one counter group per run) for the C2, C3, C4
# and C5 bench workloads; summarise here with scripts/pmc_summary.py TAG_<cfg> <cfg> W.
TAG=${1:-r02}
SET_A="SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAVE_CYCLES"
BENCH_ARGS="--config C2 --kernel-samples 20" bash scripts/pmc.sh ${TAG}_C2 "$SET_A" "FETCH_SIZE" "WRITE_SIZE" || exit $?
BENCH_ARGS="--config C4 --steps 10 --warmup 2 --kernel-samples 10" bash scripts/pmc.sh ${TAG}_C4 "$SET_A" "FETCH_SIZE" "WRITE_SIZE" || exit $?
BENCH_ARGS="--config C3 --steps 5 --warmup 2 --kernel-samples 5" bash scripts/pmc.sh ${TAG}_C3 "$SET_A" "FETCH_SIZE" "WRITE_SIZE" || exit $?
BENCH_ARGS="--config C5 --steps 10 --warmup 2 --kernel-samples 10" bash scripts/pmc.sh ${TAG}_C5 "$SET_A" "FETCH_SIZE" "WRITE_SIZE" || exit $?
