# r02o: k_apply syndrome prefetch depth (RQHIP_APPLY_PD 2 / 4 / 8): GPU decode tests, then the full
# encode+decode bench per depth with kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
for PD in 2 4 8; do
  RQHIP_LIB=$EXP RQHIP_APPLY_PD=$PD timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench_pd$PD.json 2> $O/bench_pd$PD.err || exit 1
  echo "pd$PD $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench_pd$PD.json)"
done
for PD in 2 4 8; do
  RQHIP_LIB=$EXP RQHIP_APPLY_PD=$PD timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof$PD -o pd$PD -- python3 bench.py --cpu-sample 0 --steps 5 > $O/prof$PD.log 2>&1 || exit 1
  grep -h "k_apply\|k_solve_fast" $O/prof$PD/*/pd${PD}_kernel_stats.csv $O/prof$PD/pd${PD}_kernel_stats.csv 2>/dev/null | cut -c1-160
done
echo DONE
