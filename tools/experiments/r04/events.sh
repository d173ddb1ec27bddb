# r04: the ~5-10 us gaps around the engine's own stream markers (workspace `last`, the side-stream `cpy`
# wait): fence-free internal events (RQHIP_EV_NOFENCE=1) against the default, interleaved bench runs,
# then kernel traces of both (experiments library).
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04f}
B='bench:--cpu-sample 0'
bash tools/experiments/run.sh $T/base1 "$B" && \
RQHIP_EV_NOFENCE=1 bash tools/experiments/run.sh $T/nf1 "$B" && \
bash tools/experiments/run.sh $T/base2 "$B" && \
RQHIP_EV_NOFENCE=1 bash tools/experiments/run.sh $T/nf2 "$B" && \
bash tools/experiments/run.sh $T/base3 "$B" && \
RQHIP_EV_NOFENCE=1 bash tools/experiments/run.sh $T/nf3 "$B" && \
bash tools/experiments/run.sh $T/pbase prof && \
RQHIP_EV_NOFENCE=1 bash tools/experiments/run.sh $T/pnf prof
