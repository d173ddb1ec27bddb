#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r01r
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "async or concurrent or batch_decode_round" -x -v --timeout 120 --timeout-method thread > gpurun_out/r01r/tests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py > gpurun_out/r01r/bench.json 2> gpurun_out/r01r/bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r01r/tl -o tl -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r01r/tl.log 2>&1 || exit 1
echo done
