# r02g: encode launch time vs IR schedule (Horner passes), and SQ counters of the chosen program.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02g
for P in 0 1 2 3 4 5 6 8; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_PASSES=$P timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 10 > gpurun_out/r02g/passes_$P.log 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/r02g/sq1 -o sq1 -- python3 tools/colbench.py 1024 1200 1100 1024 3 > gpurun_out/r02g/sq1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/r02g/sq2 -o sq2 -- python3 tools/colbench.py 1024 1200 1100 1024 3 > gpurun_out/r02g/sq2.log 2>&1
echo EXIT $?
