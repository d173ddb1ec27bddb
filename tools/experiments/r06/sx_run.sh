# Precomputed syndromes: the apply tests (both paths against k_apply), then the A/B (sx_ab.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-sx}
mkdir -p gpurun_out/$O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_apply.py tests/test_gpu_decode_limits.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/$O/pytest.log | tail -20; tail -5 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
bash tools/experiments/r06/sx_ab.sh $O
