# Round-5 checkpoint: the zero-overhead parity test's rank-deficient count, then the full check.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r05q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k zero_overhead -s -q --timeout 240 --timeout-method thread > $O/zero_overhead.log 2>&1 || { tail -20 $O/zero_overhead.log; exit 1; }
grep "rank-deficient" $O/zero_overhead.log
bash tools/experiments/r05/full_check.sh ${1:-r05q}
