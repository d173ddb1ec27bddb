# r02ba: pass count P under the balanced grid (960 waves): P=2 (default) vs 3 vs 4, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ba
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
for rep in 1 2; do
  run p2_$rep RQHIP_PASSES=2
  run p3_$rep RQHIP_PASSES=3
  run p4_$rep RQHIP_PASSES=4
done
echo DONE
