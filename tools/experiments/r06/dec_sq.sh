# SQ counters of the decode's solver and apply kernels (config 3, release library), one --pmc pass.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-dec_sq}
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --kernel-include-regex "k_solve_pq|rq_apply_gi" --output-format csv -d $O/sq -o sq -- python3 -u tools/experiments/r06/solve_ab.py 2 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
echo DONE
