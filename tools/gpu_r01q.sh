#!/bin/bash
# r01q: one-step GPU timeline of the bench (kernel + copy trace) and a k_apply slice-size sweep.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r01q
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r01q/tl -o tl -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r01q/tl.log 2>&1 || exit 1
for cap in 20 28 32 16 12; do
  RQHIP_APPLY_CAP=$cap timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r01q/cap$cap -o cap -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/r01q/cap$cap.log 2>&1 || exit 1
done
echo done
