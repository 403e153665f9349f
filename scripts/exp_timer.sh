#!/bin/bash
# kernel-duration agreement: fence-free HIP events vs torch events vs rocprof
mkdir -p gpurun_out/timer
for args in "--timer hip" "--timer torch" "--timer hip --event-every 1" "--timer torch --event-every 1"; do
  timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline $args > gpurun_out/timer/out.json 2> gpurun_out/timer/err.log
  rc=$?; if [ $rc -ne 0 ]; then echo "[$args] rc=$rc"; tail -5 gpurun_out/timer/err.log; exit $rc; fi
  python -c "import json; j=json.loads(open('gpurun_out/timer/out.json').read().strip().splitlines()[-1]); r=j['roofline']; print('[$args]', 'evals/s %.4e'%j['value'], 'ms/step %.4f'%j['ms_per_step'], 'eval %.4f prep %.4f n=%d'%(r['kernel_ms'], r['prep_kernel_ms'], r['kernel_event_samples']))"
done
