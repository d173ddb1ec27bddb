# Round-6 end measurements beside the checkpoint: the two-rank gloo rehearsal on one GPU and the
# host-memory end-to-end rate at config 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06x}
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --cpu-sample 0 > $O/bench_gpus2_gloo_one_gpu.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 300 python3 tools/e2e_host_api.py 1024 3 > $O/e2e_host_api.log 2>&1 || { tail -5 $O/e2e_host_api.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_gpus2_gloo_one_gpu.json')); print(d['value'], d['unit'], d['ms_per_step'], d['n_gpus'])"
tail -3 $O/e2e_host_api.log
echo DONE
