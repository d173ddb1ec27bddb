# r02au: balanced persistent rounds in the release library: GPU tests, bench lines (configs 3 and 2)
# and kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02au
mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
timeout -k 10 200 python3 bench.py --config 2 --cpu-sample 0 > $O/bench_cfg2.json 2>> $O/bench.err || exit 1
cat $O/bench_cfg2.json
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || exit 1
cut -c1-140 $O/prof/bench_kernel_stats.csv | head -6
echo DONE
