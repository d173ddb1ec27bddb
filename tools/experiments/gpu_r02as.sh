# r02as: allocator knobs re-swept with cached source loads (a dropped source row is now re-read
# mostly from L2): source-row victim bias, evicted source rows into LDS or not, pass count,
# look-ahead / outstanding loads.  Interleaved, two repetitions, K=1024 encode (colbench).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02as
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h -e encode -e mismatching $O/$n.log | tr '\n' ' ')"
}
for rep in 1 2; do
  run base_$rep
  run bias150_$rep RQHIP_SRC_BIAS=150
  run bias250_$rep RQHIP_SRC_BIAS=250
  run bias60_$rep RQHIP_SRC_BIAS=60
  run srclds0_$rep RQHIP_SRC_LDS=0
  run p3_$rep RQHIP_PASSES=3
  run la480_$rep RQHIP_ALLOC=250,256,480,240,56,157
  run vm40_$rep RQHIP_ALLOC=250,256,320,160,40,157
done
echo DONE
