# Perm-based solver (RQHIP_SOLVE_PM=1, experiments build): full GPU parity suite, then bench A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/solvepm2
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
RQHIP_SOLVE_PM=1 timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for v in 0 1 0 1; do
  RQHIP_SOLVE_PM=$v timeout -k 10 180 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/bench_$v.$SECONDS.json 2>/dev/null
done
RQHIP_SOLVE_PM=1 timeout -s KILL 150 rocprofv3 --kernel-include-regex solve --kernel-trace --stats --output-format csv -d $O/prof -o pm -- python tools/hostdec_trace.py 2048 1200 3 > /dev/null 2>&1
for kt in "2048 1200"; do
  RQHIP_SOLVE_PM=0 timeout -k 10 200 python tools/hostdec_trace.py $kt 5 > $O/host_pm0.log 2>&1
  RQHIP_SOLVE_PM=1 timeout -k 10 200 python tools/hostdec_trace.py $kt 5 > $O/host_pm1.log 2>&1
done
RQHIP_SOLVE_PM=0 timeout -s KILL 150 rocprofv3 --kernel-include-regex solve --kernel-trace --stats --output-format csv -d $O/prof -o fast -- python tools/hostdec_trace.py 2048 1200 3 > /dev/null 2>&1
