#!/bin/bash
# One GPU session: parity tests, smoke, C2/C3/C5 bench lines, kernel traces of the
# likelihood bench and the device sampler, PMC passes on the C2 eval kernel.
# $1 = profile tag.  Stops at the first step whose exit status is > 1.
TAG=${1:-r02}
bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/profile_dsampler.sh ${TAG}_ds || exit $?
bash scripts/gpu_pmc.sh $TAG || exit $?
