# r04: what bounds the encode column program (K=1024 config 3 unless noted)?  The single-wave program
# as shipped, at 512 resident waves, with four-row staging of its source rows (RQHIP_DMA4 quads); the
# pair with dword loads and with four-row staging in its load wave.  Parity spot check per run.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/r04d && mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 tools/colbench.py $CB > $O/$tag.log 2>&1 || { echo "$tag FAILED"; tail -5 $O/$tag.log; exit 1; }
  echo "$tag: $(grep -h mismatching $O/$tag.log | awk '{print $NF}' | tr '\n' ' ') $(grep -h encode $O/$tag.log | tail -1)"
}
CB="1024 1200 1100 16 3"
run pair4_small RQHIP_PAIR=1
run single_d4_small RQHIP_PAIR=0 RQHIP_DMA4=8
run pair_ha3_small RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,32,1200,3
CB="1024 1200 1100 1024 10"
run single RQHIP_PAIR=0
run single_d4q4 RQHIP_PAIR=0 RQHIP_DMA4=4
run single_d4q8 RQHIP_PAIR=0 RQHIP_DMA4=8
run pair_dword RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0
run pair4 RQHIP_PAIR=1
run pair4_q16 RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,16,800
run pair4_lag2 RQHIP_PAIR=1 RQHIP_PAIR_CFG=2,16,192
run pair4_ha2 RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,32,1200,2
run pair4_ha3 RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,32,1200,3
run pair4_ha4 RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,32,1200,4
run single_w512 RQHIP_PAIR=0 RQHIP_WAVES=512
run single2 RQHIP_PAIR=0
run pair4_2 RQHIP_PAIR=1
CB="2048 1200 2260 512 10"
run k2048_single RQHIP_PAIR=0
run k2048_pair4 RQHIP_PAIR=1
run k2048_d4q8 RQHIP_PAIR=0 RQHIP_DMA4=8
