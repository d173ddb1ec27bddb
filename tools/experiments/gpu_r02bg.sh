# r02bg: instruction-cache behaviour of the column program (SQC counters), bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02bg
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_INSTS_VALU --kernel-include-regex rq_colprog --output-format csv -d $O/ic -o ic -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/ic.log 2>&1 || { tail -5 $O/ic.log; exit 1; }
echo DONE
