# The solve list in decreasing erasure count (longest first): decode GPU tests, then the decode A/B and
# the bench A/B (experiments library, RQHIP_LPT=0 keeps block order).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-lpt}
mkdir -p gpurun_out/$O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_apply.py tests/test_gpu_decode_limits.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py tests/test_gpu_host_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" gpurun_out/$O/pytest.log | tail -20; exit 1; }
tail -1 gpurun_out/$O/pytest.log
REPS=20 RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so SETTINGS="RQHIP_LPT=0 RQHIP_LPT=1" bash tools/experiments/r06/sx_ab.sh $O/dec > /dev/null || exit 1
SETTINGS="RQHIP_LPT=0 RQHIP_LPT=1" bash tools/experiments/r06/sx_bench.sh $O/bench || exit 1
