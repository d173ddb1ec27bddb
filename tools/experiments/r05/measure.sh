# Round-5 HEAD measurements beside the checkpoint (gpu_quick.sh): configs 2 and 5, the end-to-end
# host-memory rate at config 3, HBM traffic of the encode launch (FETCH_SIZE /
# WRITE_SIZE passes), SQ counters + GRBM clock of the encode program
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05m}
mkdir -p $O
timeout -k 10 200 python3 bench.py --config 2 --cpu-sample 0 > $O/bench_cfg2.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench_cfg2.json
timeout -k 10 300 python3 bench.py --config 5 --cpu-sample 0 > $O/bench_cfg5.json 2>> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench_cfg5.json
timeout -k 10 300 python3 tools/e2e_host_api.py 1024 3 > $O/e2e_host_api.log 2>&1 || { tail -5 $O/e2e_host_api.log; exit 1; }
tail -5 $O/e2e_host_api.log
bash tools/gpu_profile.sh ${1:-r05m} > $O/traffic.log 2>&1 || { tail -10 $O/traffic.log; exit 1; }
cp gpurun_out/pmc_traffic/summary.json $O/traffic.json && cat $O/traffic.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex rq_colprog --output-format csv -d $O/sq -o sq -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-include-regex rq_colprog --output-format csv -d $O/sq2 -o sq -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
echo DONE
