set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfgt
timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/cfgt/test.log 2>&1 || { tail -20 gpurun_out/cfgt/test.log; exit 1; }
tail -3 gpurun_out/cfgt/test.log
bash tools/experiments/r05/gsolve.sh
