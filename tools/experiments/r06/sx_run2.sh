set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sxb2
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_apply.py tests/test_gpu_decode_limits.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/sxb2/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/sxb2/pytest.log | tail -20; exit 1; }
tail -1 gpurun_out/sxb2/pytest.log
bash tools/experiments/r06/sx_bench.sh sxb2
