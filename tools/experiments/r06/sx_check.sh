# GPU check of the precomputed-syndrome path after moving it to the experiments library: the release
# apply / decode-limit tests, then the experiments library's agreement test (RQHIP_APPLY_SX=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sxc}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_apply.py tests/test_gpu_decode_limits.py "tests/test_gpu_experimental_programs.py::test_precomputed_syndromes_agree" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error|assert" $O/pytest.log | tail -20; exit 1; }
tail -1 $O/pytest.log
