# r02ax: k_apply output-slice width KC (4/8/12/16) after the buffer-load/branch-free ring change
# (bench kernel stats, experiments library via RQHIP_LIB in the bench's rqhip import).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ax
mkdir -p $O
for KC in 8 12 4 16 8; do
  timeout -s KILL 150 env RQHIP_APPLY_KC=$KC rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc$KC -o b -- python3 tools/experiments/bench_exp.py --cpu-sample 0 > $O/kc$KC.json 2> $O/kc$KC.err || exit 1
  echo "KC=$KC $(grep -h k_apply $O/kc$KC/b_kernel_stats.csv | cut -d, -f1,4)"
done
echo DONE
