# Host decode timeline: plain timing, then kernel + memory-copy trace (no counters).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/hostdec2
timeout -k 10 200 python tools/hostdec_trace.py 512 256 4 > gpurun_out/hostdec2/plain_512_256.log 2>&1
timeout -k 10 200 python tools/hostdec_trace.py 2048 1200 4 > gpurun_out/hostdec2/plain_2048_1200.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hostdec2/tr -o run -- python tools/hostdec_trace.py 512 256 3 > gpurun_out/hostdec2/trace_512_256.log 2>&1
