set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
RQHIP_DBG=0 timeout -k 10 120 python tools/ablate.py > gpurun_out/ablate.log 2>&1 && \
RQHIP_DBG=2 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate.log 2>&1 && \
RQHIP_STAMP_FILE=gpurun_out/stamps.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
echo EXIT $?
