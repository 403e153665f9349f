# parity tests, smoke, C2 and C3 bench lines; stops on fault-like status
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-3000
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 600 python bench.py --steps 200 --warmup 20
step bench_c3 600 python bench.py --ncad 20000 --steps 20 --warmup 3 --no-cpu-baseline
step bench_c5 600 python bench.py --config C5 --steps 100 --warmup 10
