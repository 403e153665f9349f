set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 120 scripts/probes/valu_probe > gpurun_out/s1/valu_probe.log 2>&1 || exit $?
bash scripts/pmc_kernel.sh stallA "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" > gpurun_out/s1/stallA.log 2>&1 || exit $?
bash scripts/pmc_kernel.sh stallB "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU" > gpurun_out/s1/stallB.log 2>&1 || exit $?
