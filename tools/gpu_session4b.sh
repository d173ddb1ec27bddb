set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/diag_c.py > gpurun_out/diag_c.log 2>&1; echo diag rc=$? >> gpurun_out/diag_c.log
timeout -k 10 400 python -m pytest tests -m gpu -q --tb=line > gpurun_out/pytest_gpu_all.log 2>&1; echo pytest rc=$?
