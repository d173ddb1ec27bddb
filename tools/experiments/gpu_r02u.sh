# r02u: decode descriptor upload on its own copy stream (RQHIP_DEC_COPY=1) vs in stream order.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02u
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
RQHIP_LIB=$EXP RQHIP_DEC_COPY=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_limits.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for C in 0 1 0 1; do
  RQHIP_LIB=$EXP RQHIP_DEC_COPY=$C timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench_c$C.json 2> $O/bench_c$C.err || exit 1
  echo "copy$C $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench_c$C.json)"
done
echo DONE
