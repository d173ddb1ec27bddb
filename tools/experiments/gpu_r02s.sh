# r02s: per-block device zeroing (no per-row list upload) and no per-call event: GPU tests, bench,
# kernel trace (gaps between the decode kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench.json 2> $O/bench.err || exit 1
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])' $O/bench.json
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 --steps 5 > $O/prof.log 2>&1 || exit 1
echo DONE
