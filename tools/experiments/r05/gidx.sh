#!/bin/bash
# VGPR index mode vs v_perm issue rates (tools/micro/gidx_gen.py) at 1-4 waves per SIMD
set -e
cd "$(dirname "$0")/../../.."
OUT=gpurun_out/gidx; mkdir -p $OUT
python3 tools/micro/gidx_gen.py $OUT/bin > /dev/null
for W in 1 2 3 4; do
  echo "W=$W"
  GRID=$((1024 * W)) WGS=64 timeout -k 10 60 tools/micro/clockrun $OUT/bin/gidx.hsaco k_gi k_gi2 k_x2 k_sidx k_salu k_perm k_mul45
done 2>&1 | tee $OUT/gidx.txt
