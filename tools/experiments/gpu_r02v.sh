# r02v: decode without the zeroing pass (k_apply starts from the erased rows' bytes): GPU tests, bench,
# kernel trace; and the step without the async status download (experiments, timing only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02v
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench.json
RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_ASYNC_NOSTATUS=1 timeout -k 10 200 python3 bench.py --cpu-sample 0 --no-verify > $O/bench_nostatus.json 2> $O/bench_nostatus.err || { tail -5 $O/bench_nostatus.err; exit 1; }
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print("nostatus", d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench_nostatus.json
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 --steps 5 > $O/prof.log 2>&1 || exit 1
echo DONE
