# r02k: LDS-DMA source staging depth (RQHIP_LA_DMA) for the encode program, and the e <= 64
# solver at one vs four waves per block (RQHIP_SOLVE_NW) in the full encode+decode bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
run base
for D in 400 800 1500 3000; do run dma$D RQHIP_LA_DMA=$D; done
run dma1500_lds200 RQHIP_LA_DMA=1500 RQHIP_ALLOC=0,0,0,0,0,201
for NW in 4 1; do
  RQHIP_LIB=$EXP RQHIP_SOLVE_NW=$NW timeout -k 10 200 python3 bench.py --cpu-sample 0 > $O/bench_nw$NW.json 2> $O/bench_nw$NW.err || exit 1
  echo "nw$NW $(cat $O/bench_nw$NW.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["config"]["encode_ms"], d["config"]["decode_ms"])')"
done
RQHIP_LIB=$EXP RQHIP_SOLVE_NW=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/prof -o nw1 -- python3 bench.py --cpu-sample 0 --steps 5 > $O/prof.log 2>&1 || exit 1
echo DONE
