# r02ar: SQ counters of the decode solver (register-resident k_solve_pm) over the bench workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ar
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-include-regex k_solve_pm --output-format csv -d $O/sq1 -o sq1 -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES --kernel-include-regex k_solve_pm --output-format csv -d $O/sq2 -o sq2 -- python3 bench.py --cpu-sample 0 --steps 3 --warmup 1 > $O/sq2.log 2>&1 || exit 1
echo DONE
