# r04: kernel-boundary costs in the bench step.  A kernel that leaves B bytes dirty in L2 pays ~B / 6 TB/s
# at the next dependent boundary (MI355X_MICROARCH.md, boundary row): the encode's 93 MB of repairs and
# the decode's 93 MB of r0 are written `nt` (kept in L2).  Output-store policies of the column program
# (RQHIP_POLICY "src;out;scr_st;scr_ld"), and the descriptor wait before the syndrome program
# (RQHIP_DESC_WAIT=1).  Interleaved bench runs (experiments library), then kernel traces of two.
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04e}
B='bench:--cpu-sample 0'
RQHIP_POLICY=";nt;;sc1" bash tools/experiments/run.sh $T/base1 "$B" && \
RQHIP_POLICY=";sc1;;sc1" bash tools/experiments/run.sh $T/sc1_1 "$B" && \
RQHIP_POLICY=";sc0 sc1;;sc1" bash tools/experiments/run.sh $T/sc01_1 "$B" && \
RQHIP_POLICY=";nt sc1;;sc1" bash tools/experiments/run.sh $T/ntsc1_1 "$B" && \
RQHIP_DESC_WAIT=1 bash tools/experiments/run.sh $T/wait1 "$B" && \
RQHIP_POLICY=";nt;;sc1" bash tools/experiments/run.sh $T/base2 "$B" && \
RQHIP_POLICY=";sc1;;sc1" bash tools/experiments/run.sh $T/sc1_2 "$B" && \
RQHIP_POLICY=";sc0 sc1;;sc1" bash tools/experiments/run.sh $T/sc01_2 "$B" && \
RQHIP_POLICY=";nt sc1;;sc1" bash tools/experiments/run.sh $T/ntsc1_2 "$B" && \
RQHIP_DESC_WAIT=1 bash tools/experiments/run.sh $T/wait2 "$B" && \
RQHIP_POLICY=";sc1;;sc1" RQHIP_APPLY_SC1=1 bash tools/experiments/run.sh $T/allsc1_1 "$B" && \
RQHIP_POLICY=";nt;;sc1" bash tools/experiments/run.sh $T/pbase prof && \
RQHIP_POLICY=";sc1;;sc1" RQHIP_APPLY_SC1=1 bash tools/experiments/run.sh $T/psc1 prof
