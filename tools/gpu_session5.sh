set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_c.py > gpurun_out/diag_c.log 2>&1 && \
timeout -k 10 400 python -m pytest tests -m gpu -q --tb=short -x > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python tools/ablate.py > gpurun_out/ablate5.log 2>&1 && \
RQHIP_PASSB=1 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate5.log 2>&1 && \
RQHIP_WAVES=16 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate5.log 2>&1 && \
RQHIP_WAVES=16 RQHIP_PASSB=1 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate5.log 2>&1 && \
timeout -k 10 200 python tools/micro/interp_bench.py > gpurun_out/interp_v3.log 2>&1 && \
RQHIP_STAMP_FILE=gpurun_out/stamps_v3.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate5.log 2>&1 && \
RQHIP_PASSB=1 RQHIP_STAMP_FILE=gpurun_out/stamps_v3_pb1.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate5.log 2>&1
echo EXIT $?
