# r02ak: column programs in multi-wave workgroups (RQHIP_WGW waves of one CU take consecutive
# items): GPU tests at the release default (4), then an interleaved A/B of W = 1/2/4/8 at K=1024 and
# K=256, then the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ak
mkdir -p $O
timeout -k 10 120 python3 tools/experiments/perobj_check.py > $O/perobj.log 2>&1 && tail -1 $O/perobj.log && timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, K, N, env...
  local n=$1 K=$2 N=$3; shift 3
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py $K 1200 $N 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h -e encode -e mismatching $O/$n.log | tr '\n' ' ')"
}
for rep in 1 2; do
  for W in 1 4 2 8; do run k1024_${rep}_w$W 1024 1100 RQHIP_WGW=$W; done
done
for W in 1 4 2; do run k256_w$W 256 282 RQHIP_WGW=$W; done
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
echo DONE
