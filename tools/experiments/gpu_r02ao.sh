# r02ao: solver row gather with sixteen loads in flight: decode GPU tests, kernel stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ao
mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || exit 1
cat $O/prof_bench.json
cut -c1-140 $O/prof/bench_kernel_stats.csv | head -8
echo DONE
