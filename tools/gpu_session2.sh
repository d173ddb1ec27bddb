set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
RQHIP_WAVES=16 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu16.log 2>&1 && \
timeout -k 10 200 python tools/micro/interp_bench.py > gpurun_out/interp8.log 2>&1 && \
RQHIP_WAVES=16 timeout -k 10 200 python tools/micro/interp_bench.py > gpurun_out/interp16.log 2>&1 && \
RQHIP_WAVES=16 timeout -k 10 120 python tools/ablate.py > gpurun_out/ablate16.log 2>&1 && \
RQHIP_WAVES=16 RQHIP_STAMP_FILE=gpurun_out/stamps16.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate16.log 2>&1
echo EXIT $?
