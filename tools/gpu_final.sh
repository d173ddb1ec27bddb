# Round checkpoint on one MI355X: every GPU test, smoke, the bench line (config 3 with the CPU
# baseline), configs 2 and 5, rocprofv3 kernel stats of the bench, HBM traffic of the encode launch
# (separate FETCH_SIZE / WRITE_SIZE passes), SQ counters of the encode program.  Usage: gpu_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02z}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python3 bench.py --config 2 --cpu-sample 0 > $O/bench_cfg2.json 2>> $O/bench.err || exit 1
timeout -k 10 300 python3 bench.py --config 5 --cpu-sample 0 > $O/bench_cfg5.json 2>> $O/bench.err || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || exit 1
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
bash tools/gpu_profile.sh $TAG > $O/traffic.log 2>&1 || exit 1
cp gpurun_out/pmc_traffic/summary.json $O/traffic.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex rq_colprog --output-format csv -d $O/sq -o sq -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/sq.log 2>&1 || exit 1
echo DONE
