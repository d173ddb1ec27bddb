# r02aw: SQ counters of k_apply over the bench workload (where its issue slots go).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02aw
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --kernel-include-regex k_apply --output-format csv -d $O/sq1 -o sq1 -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD --kernel-include-regex k_apply --output-format csv -d $O/sq2 -o sq2 -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/sq2.log 2>&1 || exit 1
echo DONE
