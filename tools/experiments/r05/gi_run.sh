cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gi1
timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -v --timeout 120 --timeout-method thread > gpurun_out/gi1/test_apply.log 2>&1
rc=$?
echo "pytest rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/experiments/r05/apply_ab.py 10 > gpurun_out/gi1/ab.log 2>&1
