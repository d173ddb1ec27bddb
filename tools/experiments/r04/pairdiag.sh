# r04: what holds the pair back?  Diagnostic builds (RQHIP_DIAG, wrong bytes, timing only): the pair
# without its barriers (128: the waves run decoupled), without XOR work (32), without source loads (4),
# and combinations, against the single wave with the same diagnostics.  K=1024 config 3, colbench.
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04i}
C='col:1024,1200,1100,1024,10'
P="RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0"
run() { local tag=$1; shift; env "$@" bash tools/experiments/run.sh $T/$tag "$C" | grep encode | sed "s/^/$tag: /"; }
run pair          RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0 && \
run pair_nobar    RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0 RQHIP_DIAG=128 && \
run pair_noxor    RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0 RQHIP_DIAG=32 && \
run pair_noload   RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0 RQHIP_DIAG=4 && \
run pair_nobar_noxor RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0 RQHIP_DIAG=160 && \
run pair_nobar_noload RQHIP_PAIR=1 RQHIP_PAIR_CFG=6,16,192,0 RQHIP_DIAG=132 && \
run single        RQHIP_PAIR=0 && \
run single_noxor  RQHIP_PAIR=0 RQHIP_DIAG=32 && \
run single_noload RQHIP_PAIR=0 RQHIP_DIAG=4 && \
run pair_staged   RQHIP_PAIR=1 && \
run pair_staged_nobar RQHIP_PAIR=1 RQHIP_DIAG=128
