# Round-1 measurement session: parity, bench line, rocprofv3 kernel trace + HBM counters.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q --tb=short -x > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_encode --output-format csv -d gpurun_out/prof_fetch -o fetch -- python3 tools/ablate.py > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_encode --output-format csv -d gpurun_out/prof_write -o write -- python3 tools/ablate.py > gpurun_out/prof_write.log 2>&1 && \
RQHIP_DBG=6 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_encode --output-format csv -d gpurun_out/prof_fetch_cal -o cal -- python3 tools/ablate.py > gpurun_out/prof_fetch_cal.log 2>&1
echo EXIT $?
