# r02az: decode solver beside the syndrome program on CU-masked internal streams (RQHIP_SOLVE_SIDE=1)
# against the in-stream order (0), interleaved, experiments library; the bench verifies every block.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02az
mkdir -p $O
for rep in 1 2; do
  for SIDE in 0 1; do
    n=side${SIDE}_$rep
    env RQHIP_SOLVE_SIDE=$SIDE timeout -k 10 200 python3 tools/experiments/bench_exp.py --cpu-sample 0 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
    python3 -c "import json;b=json.load(open('$O/$n.json'));print('$n', b['value'], b['config']['encode_ms'], b['config']['decode_ms'])"
  done
done
env RQHIP_SOLVE_SIDE=1 timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b -- python3 tools/experiments/bench_exp.py --cpu-sample 0 > $O/prof.json 2> $O/prof.err || exit 1
cut -c1-120 $O/prof/b_kernel_stats.csv | head -6
echo DONE
