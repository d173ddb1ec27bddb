#!/bin/bash
# Bench variants in one box, 2 rounds: each argument is "ENV=VAL ... -- bench args" (env may be empty).
set -o pipefail
mkdir -p gpurun_out/ab
: > gpurun_out/ab/abn.log
for i in 1 2; do
  for v in "$@"; do
    echo "V $v" >> gpurun_out/ab/abn.log
    envs="${v%%--*}"; args="${v#*--}"
    env $envs timeout -k 10 120 python bench.py --cpu-sample 0 $args >> gpurun_out/ab/abn.log 2>/dev/null || exit 1
  done
done
echo done
