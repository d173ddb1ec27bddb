cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/spmc; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --kernel-include-regex "k_solve_pq|rq_apply_gi" --output-format csv -d $O/a -o a -- python3 tools/experiments/r05/apply_ab.py 1 > $O/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_solve_pq|rq_apply_gi" --output-format csv -d $O/b -o b -- python3 tools/experiments/r05/apply_ab.py 1 > $O/b.log 2>&1 || exit 1
