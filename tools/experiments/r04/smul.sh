# r04: the encode program's lgkmcnt(0) per 16 source loads (the scalar row-offset window; it also drains
# the LDS operations in flight) against an s_mul per load (RQHIP_SRC_SMUL=1).  Interleaved colbench runs
# at config 3 and the SQ counters of both (experiments library).
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04g}
C='col:1024,1200,1100,1024,10'
bash tools/experiments/run.sh $T/base1 "$C" && \
RQHIP_SRC_SMUL=1 bash tools/experiments/run.sh $T/smul1 "$C" && \
bash tools/experiments/run.sh $T/base2 "$C" && \
RQHIP_SRC_SMUL=1 bash tools/experiments/run.sh $T/smul2 "$C" && \
bash tools/experiments/run.sh $T/base3 "$C" && \
RQHIP_SRC_SMUL=1 bash tools/experiments/run.sh $T/smul3 "$C" && \
bash tools/experiments/run.sh $T/sqbase sq && \
RQHIP_SRC_SMUL=1 bash tools/experiments/run.sh $T/sqsmul sq
