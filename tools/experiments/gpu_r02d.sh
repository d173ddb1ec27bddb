set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fecquic.py tests/test_gpu_host_batch.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r02d_pytest.log 2>&1
