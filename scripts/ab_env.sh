#!/bin/bash
# interleaved A/B of environment settings on one bench workload:
#   bash scripts/ab_env.sh "<bench args>" "ENV1=a ENV2=b" "ENV1=c" ...
ARGS=$1; shift
for rnd in 1 2 3; do
  for e in "$@"; do
    r=$(env $e timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 $ARGS 2>/dev/null | tail -1 | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(f\"{j['ms_per_step']:.4f} ms/step  {j['value']:.3e}\")") || exit 1
    echo "[$e] $r"
  done
done
