#!/bin/bash
# PMC counters of the eval kernel for each lib/variants/*.so (kernel-trace only;
# one --pmc pass per variant and counter set).  Summary: scripts/pmc_ab_summary.py
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SETS=${PMC_SETS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM"}
for lib in $R/hb_mcmc_amd/lib/variants/libhbmi_*.so; do
  tag=$(basename $lib .so)
  i=0
  for set in $SETS; do :; done
  IFS='|' read -ra arr <<< "$SETS"
  for set in "${arr[@]}"; do
    i=$((i+1))
    HBMI_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $OUT/${tag}_$i -o run \
      -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --sampler-iters 0 --kernel-samples 5 ${BENCH_ARGS} > $OUT/${tag}_$i.log 2>&1
    rc=$?; echo "$tag set $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/${tag}_$i.log; exit $rc; fi
  done
done
python3 $R/scripts/pmc_ab_summary.py $OUT
