# r04 check on one MI355X: every GPU test (product library), the bench line, the host enqueue probe,
# and the two-rank gloo rehearsal of bench.py (both ranks on the one GPU).
cd $GRAFT_REPO_ROOT
T=${1:-r04c}
bash tools/experiments/run.sh $T tests bench py:"tools/experiments/probes.py:host_enqueue" && \
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --cpu-sample 0 > gpurun_out/$T/gloo2.json 2> gpurun_out/$T/gloo2.err && \
cat gpurun_out/$T/gloo2.json && echo CHECK DONE
