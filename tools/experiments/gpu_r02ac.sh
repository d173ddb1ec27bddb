# r02ac: residency search for on-chip programs (2/4/8 waves per SIMD): all GPU tests, config 2, small-K
# encode launches, per-object latency, the K=1024 bench (unchanged program).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ac
mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 bench.py --config 2 --cpu-sample 0 > $O/cfg2.json 2> $O/cfg2.err || exit 1
echo "cfg2 $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["roofline"]["launch_ms"])' $O/cfg2.json)"
for KN in "128 1200 148" "256 1200 282" "512 1200 571" "64 1200 80" "26 1500 32"; do
  set -- $KN
  timeout -k 10 120 python3 tools/colbench.py $1 $2 $3 1024 20 > $O/cb_$1.log 2>&1 || exit 1
  echo "K=$1 $(grep -h -e 'encode K' $O/cb_$1.log)"
done
timeout -k 10 300 python3 tools/perobj_latency.py 50 > $O/perobj_latency.json 2> $O/perobj.err || exit 1
timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench.json
timeout -k 10 300 python3 bench.py --config 5 --cpu-sample 0 > $O/cfg5.json 2> $O/cfg5.err || exit 1
echo "cfg5 $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"])' $O/cfg5.json)"
echo DONE
