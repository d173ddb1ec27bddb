set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ablate4.log
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for cfg in "8 0" "16 0" "8 1" "16 1"; do set -- $cfg
  RQHIP_WAVES=$1 RQHIP_PASSB=$2 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate4.log 2>&1 || exit 1
  echo "waves=$1 passb=$2" >> gpurun_out/ablate4.log
done
RQHIP_PASSB=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_gpu_passb1.log 2>&1 || { echo PYTEST_PASSB_FAIL; exit 1; }
timeout -k 10 200 python tools/micro/interp_bench.py > gpurun_out/interp_v3.log 2>&1 || exit 1
RQHIP_STAMP_FILE=gpurun_out/stamps_v3.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate4.log 2>&1 || exit 1
RQHIP_PASSB=1 RQHIP_STAMP_FILE=gpurun_out/stamps_v3_pb1.txt B=256 timeout -k 10 120 python tools/ablate.py >> gpurun_out/ablate4.log 2>&1
echo EXIT $?
