#!/bin/bash
# prep workgroup size A/B (HB_PREP_WMAX=16: 16 walkers per workgroup always) on C4 and C5, after the
# catalog / parity tests
set -o pipefail
O=gpurun_out/prepab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_catalog.py tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do for v in w64 w16; do for c in C4 C5; do
  envs=""; [ $v = w16 ] && envs="HB_PREP_WMAX=16"
  env $envs timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 10 --no-cpu-baseline --sampler-iters 0 --dropin-iters 0 > $O/${c}_${v}_$r.json 2> $O/${c}_${v}_$r.err || { tail -5 $O/${c}_${v}_$r.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2],sys.argv[3],round(d['value']/1e6,2),'Mevals/s',round(d['ms_per_step']*1e3,1),'us/step prep',r.get('prep_kernel_ms'))" $O/${c}_${v}_$r.json $c $v
done; done; done
