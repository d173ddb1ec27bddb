# r02j: where the encode launch time goes -- diagnostic variants (RQHIP_DIAG: 1 no global scratch,
# 2 no LDS spills, 4 no source loads, 8 no output stores), look-ahead variants, SQ counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
run base
for D in 1 2 4 8 3 7 15; do run diag$D RQHIP_DIAG=$D; done
run la480 RQHIP_ALLOC=0,0,480,0,0,0
run la640_r320 RQHIP_ALLOC=0,0,640,320,60,0
run la200 RQHIP_ALLOC=0,0,200,0,0,0
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS --kernel-include-regex rq_colprog --output-format csv -d $O/sq1 -o sq1 -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/sq1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex rq_colprog --output-format csv -d $O/sq2 -o sq2 -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/sq2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_LEVEL_WAVES SQ_WAVES --kernel-include-regex rq_colprog --output-format csv -d $O/sq3 -o sq3 -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/sq3.log 2>&1 || exit 1
echo DONE
