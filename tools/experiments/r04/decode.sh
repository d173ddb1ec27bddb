# r04 decode: the solve beside the syndrome program (RQHIP_SOLVE_BESIDE) against after it, two
# interleaved rounds; kernel stats of each; k_apply HBM traffic (FETCH/WRITE passes); the host enqueue
# probe.  Experiments library.
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04b}
RQHIP_SOLVE_BESIDE=0 bash tools/experiments/run.sh $T/off1 bench:"--cpu-sample 0" && \
RQHIP_SOLVE_BESIDE=1 bash tools/experiments/run.sh $T/on1 bench:"--cpu-sample 0" && \
RQHIP_SOLVE_BESIDE=0 bash tools/experiments/run.sh $T/off2 bench:"--cpu-sample 0" && \
RQHIP_SOLVE_BESIDE=1 bash tools/experiments/run.sh $T/on2 bench:"--cpu-sample 0" && \
RQHIP_SOLVE_BESIDE=1 bash tools/experiments/run.sh $T/onp prof && \
bash tools/experiments/run.sh $T/apply bytes && \
bash tools/experiments/run.sh $T/probe py:"tools/experiments/probes.py:host_enqueue"
