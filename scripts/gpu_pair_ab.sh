#!/bin/bash
# GPU tests, then C5 / N = 1861 bench A/B of the pair-of-waves plan for
# N = 1025..2048 against one wave of 32 cadences per lane (HB_NO_PAIR=1).
# Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out/pair
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
  > gpurun_out/pair/pytest.log 2>&1 || { tail -30 gpurun_out/pair/pytest.log; exit 1; }
tail -2 gpurun_out/pair/pytest.log
for r in 1 2; do
  for v in pair nopair; do
    envs=""; [ $v = nopair ] && envs="HB_NO_PAIR=1"
    env $envs timeout -k 10 200 python bench.py --config C5 --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 \
      --dropin-iters 0 > gpurun_out/pair/c5_${v}_$r.json 2> gpurun_out/pair/c5_${v}_$r.err || { tail -5 gpurun_out/pair/c5_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],'C5',d['value'],d['ms_per_step'])" gpurun_out/pair/c5_${v}_$r.json $v
  done
done
