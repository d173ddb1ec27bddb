# k_solve_pm with log-indexed table LUT (RQHIP_SOLVE_LUT=1, experiments build): full GPU parity
# suite, bench A/B against k_solve_pm, the wide pass at K=2048.
set -e
export TMPDIR=/tmp
O=gpurun_out/solvelut
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
RQHIP_SOLVE_LUT=1 timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for v in 0 1 0 1; do
  RQHIP_SOLVE_LUT=$v timeout -k 10 180 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/bench_$v.$SECONDS.json 2>/dev/null
done
for v in 0 1; do
  RQHIP_SOLVE_LUT=$v timeout -s KILL 150 rocprofv3 --kernel-include-regex solve --kernel-trace --stats --output-format csv -d $O/prof -o b$v -- python bench.py --steps 5 --cpu-sample 0 > /dev/null 2>&1
  RQHIP_SOLVE_LUT=$v timeout -s KILL 150 rocprofv3 --kernel-include-regex solve --kernel-trace --stats --output-format csv -d $O/prof -o w$v -- python tools/hostdec_trace.py 2048 1200 3 > /dev/null 2>&1
done
