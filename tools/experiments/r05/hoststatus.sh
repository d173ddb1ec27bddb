# Async decode statuses written by k_solve into the caller's pinned array (no status download): decode
# GPU tests, the bench, and a kernel trace of the bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-hst}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_apply.py tests/test_gpu_decode_limits.py tests/test_gpu_edge.py tests/test_gpu_streams.py -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { echo tests failed; tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; exit 1; }
echo DONE
