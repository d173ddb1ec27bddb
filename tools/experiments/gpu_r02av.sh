# r02av: concurrency of the column program: the resident cap (RQHIP_WAVES) at balanced rounds --
# 1024 -> 960 waves x 5 rounds, 800 x 6, 688 x 7, 600 x 8, 480 x 10 (fewer waves = a smaller scratch
# footprint per XCD L2 and less HBM contention).  K=1024 encode (colbench), twice, interleaved; then
# K=256 at 2 waves per SIMD (resident 2048).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02av
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, K, N, env...
  local n=$1 K=$2 N=$3; shift 3
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py $K 1200 $N 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h -e encode -e mismatching $O/$n.log | tr '\n' ' ')"
}
for rep in 1 2; do
  for W in 1024 800 688 600 480; do run k1024_w${W}_$rep 1024 1100 RQHIP_WAVES=$W; done
done
for W in 2048 1600 1200 960; do run k256_w$W 256 282 RQHIP_WAVES=$W; done
echo DONE
