#!/bin/bash
# single-context bench at N = 1100 / 1500 / 1861 / 2048, 4096 walkers, pair
# plan vs one wave of 32 cadences per lane (HB_NO_PAIR=1), interleaved
mkdir -p gpurun_out/pairn
for n in 1100 1500 1861 2048; do
  for v in pair nopair; do
    envs=""; [ $v = nopair ] && envs="HB_NO_PAIR=1"
    env $envs timeout -k 10 120 python bench.py --ncad $n --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 \
      --dropin-iters 0 > gpurun_out/pairn/n${n}_$v.json 2> gpurun_out/pairn/n${n}_$v.err || { tail -5 gpurun_out/pairn/n${n}_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],sys.argv[3],round(d['value']/1e6,2),'Mevals/s eval',round(r['kernel_ms']*1e3,1),'us')" gpurun_out/pairn/n${n}_$v.json $n $v
  done
done
