# r02at: the persistent grid's last partial round.  1024 blocks = 4 800 items over 1 024 waves (704
# waves take a fifth item); capped grids of 960 (5 items each) and 896 waves; 1092 blocks = 5 120 items
# (5 full rounds) for the per-block rate without a partial round.  K=1024 encode (colbench).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02at
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, blocks, env...
  local n=$1 B=$2; shift 2
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 $B 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
for rep in 1 2; do
  run b1024_w1024_$rep 1024
  run b1024_w960_$rep 1024 RQHIP_WAVES=960
  run b1024_w896_$rep 1024 RQHIP_WAVES=896
  run b1092_w1024_$rep 1092
  run b2048_w1024_$rep 2048
done
echo DONE
