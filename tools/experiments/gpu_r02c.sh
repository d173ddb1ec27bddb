# r02c: bench (config 3 default, config 2, config 5), rocprofv3 kernel stats of the default bench,
# PMC FETCH/WRITE traffic passes of the encode launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02c
timeout -k 10 300 python bench.py > gpurun_out/r02c/bench.json 2> gpurun_out/r02c/bench.err && \
timeout -k 10 200 python bench.py --config 2 > gpurun_out/r02c/bench_cfg2.json 2> gpurun_out/r02c/bench_cfg2.err && \
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/r02c/bench_cfg5.json 2> gpurun_out/r02c/bench_cfg5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02c/prof -o bench -- python3 bench.py > gpurun_out/r02c/prof_bench.json 2> gpurun_out/r02c/prof.err && \
bash tools/gpu_profile.sh r02 > gpurun_out/r02c/traffic.log 2>&1
echo EXIT $?
