# r04: the lean one-wave solver (k_solve_lean, RQHIP_SOLVE_LEAN=1): the decode GPU tests on it, then
# interleaved bench runs against k_solve_pq, alone and beside the syndrome program (RQHIP_SOLVE_BESIDE=1),
# and kernel traces (experiments library).
cd $GRAFT_REPO_ROOT
export LIB=exp TMPDIR=/tmp
T=${1:-r04j}
O=gpurun_out/$T && mkdir -p $O
RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_SOLVE_LEAN=1 timeout -k 10 400 python3 -u -m pytest \
  tests/test_gpu_parity.py tests/test_gpu_decode_limits.py tests/test_gpu_configs.py tests/test_gpu_edge.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_lean.log 2>&1 || { echo LEAN TESTS FAILED; tail -30 $O/pytest_lean.log; exit 1; }
tail -1 $O/pytest_lean.log
B='bench:--cpu-sample 0'
bash tools/experiments/run.sh $T/pq1 "$B" && \
RQHIP_SOLVE_LEAN=1 bash tools/experiments/run.sh $T/lean1 "$B" && \
RQHIP_SOLVE_LEAN=1 RQHIP_SOLVE_BESIDE=1 bash tools/experiments/run.sh $T/leanb1 "$B" && \
bash tools/experiments/run.sh $T/pq2 "$B" && \
RQHIP_SOLVE_LEAN=1 bash tools/experiments/run.sh $T/lean2 "$B" && \
RQHIP_SOLVE_LEAN=1 RQHIP_SOLVE_BESIDE=1 bash tools/experiments/run.sh $T/leanb2 "$B" && \
RQHIP_SOLVE_LEAN=1 bash tools/experiments/run.sh $T/plean prof && \
RQHIP_SOLVE_LEAN=1 RQHIP_SOLVE_BESIDE=1 bash tools/experiments/run.sh $T/pleanb prof
