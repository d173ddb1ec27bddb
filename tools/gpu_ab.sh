#!/bin/bash
# A/B of two bench.py argument sets in one box: A B A B A B, one JSON line each.
set -o pipefail
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.log
for i in 1 2 3; do
  echo "A $1" >> gpurun_out/ab/ab.log
  timeout -k 10 120 python bench.py --cpu-sample 0 $1 >> gpurun_out/ab/ab.log 2>/dev/null || exit 1
  echo "B $2" >> gpurun_out/ab/ab.log
  timeout -k 10 120 python bench.py --cpu-sample 0 $2 >> gpurun_out/ab/ab.log 2>/dev/null || exit 1
done
echo done
