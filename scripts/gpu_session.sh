#!/bin/bash
# One GPU session: PMC passes of C2/C3/C4/C5 summarised on the box (the counter
# file keyed by kernel build, copied to gpurun_out/profiles_new/), then parity
# tests, smoke, C2/C3/C5 bench lines (quoting those counters), kernel traces
# of the likelihood bench and of the device sampler.  $1 = profile tag.
# Stops at the first step whose exit status is > 1.
TAG=${1:-r02}
bash scripts/gpu_pmc_all.sh $TAG || exit $?
mkdir -p gpurun_out/profiles_new
python3 scripts/pmc_summary.py ${TAG}_C2 C2 4096 1024 > gpurun_out/pmc_summary_C2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py ${TAG}_C3 C3 4096 20000 > gpurun_out/pmc_summary_C3.log 2>&1 || exit $?
python3 scripts/pmc_summary.py ${TAG}_C5 C5 16384 > gpurun_out/pmc_summary_C5.log 2>&1 || exit $?
python3 scripts/pmc_summary.py ${TAG}_C4 C4 8192 1024 > gpurun_out/pmc_summary_C4.log 2>&1 || exit $?
cp profiles/pmc_counters.json profiles/${TAG}_C?_pmc_C?.json gpurun_out/profiles_new/
bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/profile_dsampler.sh ${TAG}_ds || exit $?
