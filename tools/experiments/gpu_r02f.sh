# r02f: multi-pass column programs: GPU tests, bench, kernel stats, traffic passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02f/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r02f/bench.json 2> gpurun_out/r02f/bench.err && \
timeout -k 10 200 python bench.py --config 2 --cpu-sample 0 > gpurun_out/r02f/bench_cfg2.json 2>> gpurun_out/r02f/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02f/prof -o bench -- python3 bench.py --cpu-sample 0 > gpurun_out/r02f/prof_bench.json 2> gpurun_out/r02f/prof.err && \
bash tools/gpu_profile.sh r02f > gpurun_out/r02f/traffic.log 2>&1
echo EXIT $?
