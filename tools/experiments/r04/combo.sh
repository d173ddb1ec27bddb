# r04 checkpoint + experiments in one box session: HEAD GPU tests, bench line, kernel stats of the
# bench, encode traffic PMC passes; then the encode memory-path experiments (mlp.sh).
cd $GRAFT_REPO_ROOT
TAG=${1:-r04a}
bash tools/gpu_quick.sh $TAG && \
bash tools/gpu_profile.sh $TAG > gpurun_out/$TAG/traffic.log 2>&1 && cp gpurun_out/pmc_traffic/summary.json gpurun_out/$TAG/traffic.json && \
echo TRAFFIC OK && bash tools/experiments/r04/mlp.sh
