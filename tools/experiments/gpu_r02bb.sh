# r02bb: k_apply occupancy capped by dynamic LDS (RQHIP_APPLY_LDS: 0 = VGPR-limited ~3 waves per SIMD,
# 20480 = 2 per SIMD, 40960 = 1 per SIMD); bench kernel stats through the experiments library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02bb
mkdir -p $O
for L in 0 20480 40960 0; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l$L -o b -- python3 tools/experiments/bench_exp.py --cpu-sample 0 --apply-lds $L > $O/l$L.json 2> $O/l$L.err || { tail -3 $O/l$L.err; exit 1; }
  echo "LDS=$L $(grep -h k_apply $O/l$L/b_kernel_stats.csv | cut -d, -f4)"
done
echo DONE
