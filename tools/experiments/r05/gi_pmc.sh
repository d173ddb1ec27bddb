cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi4
mkdir -p $O
for sh in 8,5,2 16,6,2; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --kernel-include-regex "rq_apply_gi|k_apply" --output-format csv -d $O/a_$sh -o a -- python3 tools/experiments/r05/apply_ab.py 1 > $O/a_$sh.log 2>&1 || exit $?
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "rq_apply_gi|k_apply" --output-format csv -d $O/b_$sh -o b -- python3 tools/experiments/r05/apply_ab.py 1 > $O/b_$sh.log 2>&1 || exit $?
done
