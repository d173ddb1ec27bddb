# r04: k_solve_pq's column buffer carrying pinfo words (RQHIP_SOLVE_PF=1): the decode GPU tests on the
# product library (its pinfo gained a nonzero bit) and on the variant, interleaved bench runs, then
# where the solve's time goes (solvesteps.sh).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r04l}
O=gpurun_out/$T && mkdir -p $O
SEL="tests/test_gpu_parity.py tests/test_gpu_decode_limits.py tests/test_gpu_configs.py tests/test_gpu_edge.py"
timeout -k 10 400 python3 -u -m pytest $SEL -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_product.log 2>&1 \
  || { echo PRODUCT TESTS FAILED; tail -30 $O/pytest_product.log; exit 1; }
tail -1 $O/pytest_product.log
RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_SOLVE_PF=1 timeout -k 10 400 python3 -u -m pytest $SEL -m gpu -x -q \
  --timeout 200 --timeout-method thread > $O/pytest_pf.log 2>&1 || { echo PF TESTS FAILED; tail -30 $O/pytest_pf.log; exit 1; }
tail -1 $O/pytest_pf.log
export LIB=exp
B='bench:--cpu-sample 0'
bash tools/experiments/run.sh $T/base1 "$B" > /dev/null && \
RQHIP_SOLVE_PF=1 bash tools/experiments/run.sh $T/pf1 "$B" > /dev/null && \
bash tools/experiments/run.sh $T/base2 "$B" > /dev/null && \
RQHIP_SOLVE_PF=1 bash tools/experiments/run.sh $T/pf2 "$B" > /dev/null && \
bash tools/experiments/run.sh $T/pbase prof > /dev/null && \
RQHIP_SOLVE_PF=1 bash tools/experiments/run.sh $T/ppf prof > /dev/null && \
echo "solve base: $(grep -h k_solve_pq gpurun_out/$T/pbase/kernel_stats_1.csv | cut -d, -f1-4)" && \
echo "solve pf:   $(grep -h k_solve_pq gpurun_out/$T/ppf/kernel_stats_1.csv | cut -d, -f1-4)" && \
bash tools/experiments/r04/solvesteps.sh $T
