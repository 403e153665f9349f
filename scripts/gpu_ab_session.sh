#!/bin/bash
# A/B session for kernel changes: bitwise parity of every lib/variants/*.so
# against the first one (scripts/ab_parity.py), then interleaved eval timing
# (scripts/ablate.py).  $1 = output tag.
TAG=${1:-ab}
O=gpurun_out/$TAG
mkdir -p $O
set -o pipefail
libs=$(ls hb_mcmc_amd/lib/variants/libhbmi_*.so)
first=""
for l in $libs; do
  b=$(basename $l .so)
  HBMI_LIB=$l timeout -k 10 300 python3 scripts/ab_parity.py dump $O/$b.npz > $O/$b.dump.log 2>&1 || { echo "dump $b failed"; tail -5 $O/$b.dump.log; exit 1; }
  if [ -z "$first" ]; then first=$O/$b.npz; else python3 scripts/ab_parity.py compare $first $O/$b.npz | tee $O/$b.cmp.log | tail -1; fi
done
ABLATE_STEPS=200 timeout -k 10 600 python3 scripts/ablate.py --sampler-iters 0 --dropin-iters 0 > $O/ablate.log 2>&1 || { echo ablate failed; tail -5 $O/ablate.log; exit 1; }
cat $O/ablate.log
