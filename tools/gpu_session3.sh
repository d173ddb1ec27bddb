set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
RQHIP_SD_MAX=15 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu_sd15.log 2>&1 && \
for cfg in "8 32" "8 15" "8 10" "8 8" "16 32" "16 15"; do set -- $cfg; \
  RQHIP_WAVES=$1 RQHIP_SD_MAX=$2 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate_sd.log 2>&1 || exit 1; echo "waves=$1 sdmax=$2" >> gpurun_out/ablate_sd.log; done && \
RQHIP_STAMP_FILE=gpurun_out/stamps_h.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate_sd.log 2>&1
echo EXIT $?
