# r02r: register-resident single-wave solver (k_solve_reg) -- GPU tests, then bench with it vs the
# four-wave LDS solver (RQHIP_SOLVE_NW=4), kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
for NW in 0 4; do
  RQHIP_LIB=$EXP RQHIP_SOLVE_NW=$NW timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench_nw$NW.json 2> $O/bench_nw$NW.err || exit 1
  echo "nw$NW $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench_nw$NW.json)"
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 --steps 5 > $O/prof.log 2>&1 || exit 1
cut -d, -f1-4 $O/prof/bench_kernel_stats.csv | cut -c1-150 | head -12
echo DONE
