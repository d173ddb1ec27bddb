# The upgraded in-place first solver (experiments library, RQHIP_SOLVE_IPX=1): the decode GPU tests under
# it, then the decode A/B against the shipped k_solve_pq<1, 4>.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-ipx}
mkdir -p gpurun_out/$O
RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_SOLVE_IPX=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_apply.py tests/test_gpu_decode_limits.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error|assert" gpurun_out/$O/pytest.log | tail -20; exit 1; }
tail -1 gpurun_out/$O/pytest.log
REPS=20 RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so SETTINGS="RQHIP_SOLVE_IPX=0 RQHIP_SOLVE_IPX=1" bash tools/experiments/r06/sx_ab.sh $O/dec > /dev/null || exit 1
echo DONE
