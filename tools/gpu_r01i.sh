# Round 1 evidence: kernel trace of the bench command + PMC traffic of the encode launch.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o trace -- python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > gpurun_out/prof_trace.log 2>&1 && \
bash tools/gpu_profile.sh r01 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo EXIT $?
