# Side-stream solve variants (RQHIP_SOLVE_SIDE 0/2/3, experiments build): bench A/B and a kernel trace of 2.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/side2
L=rl-quic-raptor_amd/build_exp/librqhip.so
for v in 0 2 3 0 2 3; do
  RQHIP_LIB=$L RQHIP_SOLVE_SIDE=$v timeout -k 10 180 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/side2/bench_$v.$SECONDS.json 2> gpurun_out/side2/bench_err.log
done
RQHIP_LIB=$L RQHIP_SOLVE_SIDE=2 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/side2/trace2 -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > /dev/null 2>&1
RQHIP_LIB=$L RQHIP_SOLVE_SIDE=3 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/side2/trace3 -o run -- python bench.py --steps 5 --warmup 2 --cpu-sample 0 > /dev/null 2>&1
