# Host-memory pipeline (3 stages, PCIe-sized chunks, deferred collect, direct scatter): parity,
# timing and traces per K, config 5.
set -e
export TMPDIR=/tmp
O=gpurun_out/hostdec8
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_host_batch.py tests/test_gpu_fecquic.py tests/test_gpu_parity.py tests/test_cpp_api.py > $O/pytest.log 2>&1
for kt in "512 256" "2048 1200" "2048 256"; do
  timeout -k 10 200 python tools/hostdec_trace.py $kt 4 >> $O/plain.log 2>&1
done
timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 > $O/cfg5.json 2> $O/cfg5.err
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- python tools/hostdec_trace.py 2048 1200 3 > $O/trace_2048_1200.log 2>&1
