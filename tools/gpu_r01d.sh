# Round 1: decode solve/apply rewrite check, bench, allocator sweep, SQ stall counters on encode.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_trace.log 2>&1 && \
for o in "251,256,320,160,56" "251,256,640,320,60" "251,256,160,80,40" "251,256,1000,500,60" "200,200,320,160,56"; do
  echo "== RQHIP_ALLOC=$o" >> gpurun_out/sweep.log
  RQHIP_ALLOC=$o timeout -k 10 120 python -u tools/colbench.py 1024 1200 1100 1024 10 >> gpurun_out/sweep.log 2>&1 || exit 3
done && \
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 ; \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/pmc_sq -o sq -- python3 tools/colbench.py 1024 1200 1100 1024 3 > gpurun_out/pmc_sq.log 2>&1
echo EXIT $?
