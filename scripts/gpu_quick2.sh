#!/bin/bash
# parity (all -m gpu tests) + C2 / C5 bench lines of the default build
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 8 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --dropin-iters 0 --sampler-iters 100 > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('C2', j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['prep_kernel_ms'], j.get('sampler_end_to_end',{}).get('device_loop'))"
timeout -k 10 300 python bench.py --config C5 --steps 100 --warmup 10 --no-cpu-baseline --dropin-iters 0 --sampler-iters 0 > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('C5', j['value'], j['ms_per_step'])"
