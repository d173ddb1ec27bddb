# Status template copied by the first solver (no per-call status upload) and fence-free staging
# events: full GPU suite, bench x3, kernel trace of the bench (gaps between launches).
set -e
export TMPDIR=/tmp
O=gpurun_out/status
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > $O/bench_$i.json 2>/dev/null
done
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o b -- python bench.py --cpu-sample 0 > /dev/null 2>&1
