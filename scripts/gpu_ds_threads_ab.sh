#!/bin/bash
# Interleaved device-loop iteration rate (scripts/sampler_rate.py --device)
# with 2 / 4 / 8 schedule producer threads (HB_DS_SCHED_THREADS)
ROUNDS=${1:-4}
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for n in 2 4 8; do
    echo -n "threads=$n $r: "
    HB_DS_SCHED_THREADS=$n timeout -k 10 120 python scripts/sampler_rate.py --device --iters 300 2>/dev/null > gpurun_out/ds_thr_rate.log
    rc=$?; tail -1 gpurun_out/ds_thr_rate.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
