#!/bin/bash
# Quick checkpoint on one MI355X: the GPU tests, the bench line, and rocprofv3 kernel stats of the bench.
# Usage: gpu_quick.sh TAG [pytest selector]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-quick}
SEL=${2:-tests}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest $SEL -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || { echo PROF rc $?; tail -5 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -12 $O/kernel_stats.csv | cut -d, -f1-8
echo DONE
