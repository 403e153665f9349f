mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
ABLATE_STEPS=20 timeout -k 10 900 python scripts/ablate.py --ncad 20000 > gpurun_out/ablate.log 2>&1; rc=$?
echo "ablate rc=$rc"; cat gpurun_out/ablate.log
ABLATE_STEPS=50 timeout -k 10 900 python scripts/ablate.py --ncad 4000 > gpurun_out/ablate2.log 2>&1; rc=$?
echo "ablate rc=$rc"; cat gpurun_out/ablate2.log
exit $rc
