# PMC passes on the encode column program (K=1024 T=1200, 1024 blocks): instruction fetch, memory.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P="python3 tools/colbench.py 1024 1200 1100 1024 3"
run() { timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/pmc/$1 -o $1 -- $P > gpurun_out/pmc/$1.log 2>&1; }
run icache "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" ; \
run ifetch "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_WAVES SQ_INSTS_SMEM" ; \
run fetch "FETCH_SIZE" ; \
run write "WRITE_SIZE" ; \
run tcc "TCC_HIT_sum TCC_MISS_sum" ; \
echo EXIT $?
