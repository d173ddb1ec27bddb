# Round-5 end measurements with the register-table apply: configs 2 and 5, the host-memory end to end,
# the two-rank gloo rehearsal on one GPU, and the apply kernel's HBM traffic (FETCH_SIZE / WRITE_SIZE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05p}
mkdir -p $O
timeout -k 10 200 python3 bench.py --config 2 --cpu-sample 0 > $O/bench_cfg2.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --config 5 --cpu-sample 0 > $O/bench_cfg5.json 2>> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 python3 tools/e2e_host_api.py 1024 3 > $O/e2e_host_api.log 2>&1 || { tail -5 $O/e2e_host_api.log; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --cpu-sample 0 > $O/bench_gpus2_gloo_one_gpu.json 2>> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rq_apply_gi --output-format csv -d $O/fetch -o f -- python3 tools/experiments/r05/apply_ab.py 1 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rq_apply_gi --output-format csv -d $O/write -o w -- python3 tools/experiments/r05/apply_ab.py 1 > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
for f in $O/bench_cfg2.json $O/bench_cfg5.json $O/bench_gpus2_gloo_one_gpu.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['unit'], d['ms_per_step'])"; done
tail -2 $O/e2e_host_api.log
echo DONE
