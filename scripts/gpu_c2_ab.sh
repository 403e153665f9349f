#!/bin/bash
# Interleaved C2 bench (eval kernel HIP-event time and evals/s) over library
# variants and environment knobs:
#   gpurun -- bash scripts/gpu_c2_ab.sh TAG ROUNDS "name=lib/variants/x.so name2=HB_X=1[,HB_Y=2] ..." ["extra bench args"]
set -o pipefail
TAG=${1:-c2ab}; ROUNDS=${2:-3}; VARS=${3:-base}; EXTRA=${4:-}
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    name=${v%%=*}; envs=""
    if [ "$v" != "$name" ]; then
      val=${v#*=}
      case "$val" in
        lib/*) envs="HBMI_LIB=$(pwd)/hb_mcmc_amd/$val" ;;
        *) envs=$(echo "$val" | tr ',' ' ') ;;
      esac
    fi
    env $envs timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 $EXTRA \
      > $O/${name}_$r.json 2> $O/${name}_$r.err || { tail -5 $O/${name}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],sys.argv[3],round(d['value']/1e6,2),'Mevals/s',round(d['ms_per_step']*1e3,2),'us/step eval',round(r['kernel_ms']*1e3,2),'us')" $O/${name}_$r.json $name $r
  done
done
