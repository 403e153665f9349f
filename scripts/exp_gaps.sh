#!/bin/bash
# launch-gap experiment: per-step events vs sampled events vs hipGraph replay
mkdir -p gpurun_out/gaps
for args in "" "--event-every 1000" "--graph" "--graph --event-every 1000"; do
  for rep in 1 2; do
    timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline $args > gpurun_out/gaps/out.json 2> gpurun_out/gaps/err.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "args=[$args] rc=$rc"; tail -5 gpurun_out/gaps/err.log; exit $rc; fi
    python -c "import json,sys; j=json.loads(open('gpurun_out/gaps/out.json').read().strip().splitlines()[-1]); print('args=[$args]', 'evals/s %.4e'%j['value'], 'ms/step %.4f'%j['ms_per_step'], 'eval %.4f prep %.4f'%(j['roofline']['kernel_ms'], j['roofline']['prep_kernel_ms']))"
  done
done
