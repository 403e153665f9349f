mkdir -p gpurun_out
timeout -k 10 900 python scripts/ablate.py $ABLATE_ARGS > gpurun_out/ablate.log 2>&1; rc=$?
echo "ablate rc=$rc"; cat gpurun_out/ablate.log
exit $rc
