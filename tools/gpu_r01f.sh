# Round 1: solve64 v2 + pinned staging check, bench, SQ issue-stall breakdown on encode.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
P="python3 tools/colbench.py 1024 1200 1100 1024 3"
run() { timeout -s KILL 90 rocprofv3 --pmc $2 --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/pmc2/$1 -o $1 -- $P > gpurun_out/pmc2/$1.log 2>&1; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_trace.log 2>&1 && \
run active "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_VALU" ; \
run fifo "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" ; \
echo EXIT $?
