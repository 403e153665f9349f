#!/bin/bash
# single-context bench, 4096 walkers: the rows kernel (lane rows over 4-16 waves) vs the block kernel (HB_NO_ROWS=1)
mkdir -p gpurun_out/rows
for n in ${NS:-3000 4001 8192 12000 16384 20000}; do
  for v in rows norows; do
    e=""; [ $v = norows ] && e="HB_NO_ROWS=1"
    env $e timeout -k 10 200 python bench.py --ncad $n --steps 20 --warmup 3 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 \
      > gpurun_out/rows/n${n}_$v.json 2> gpurun_out/rows/n${n}_$v.err || { tail -3 gpurun_out/rows/n${n}_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],sys.argv[3],round(d['value']/1e6,3),'Mevals/s',r['kernel'],round(r['kernel_ms']*1e3,1),'us')" gpurun_out/rows/n${n}_$v.json $n $v
  done
done
