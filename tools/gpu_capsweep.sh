#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/caps
for cap in "$@"; do
  RQHIP_APPLY_CAP=$cap timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/caps/cap$cap -o cap -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/caps/cap$cap.log 2>&1 || exit 1
done
echo done
