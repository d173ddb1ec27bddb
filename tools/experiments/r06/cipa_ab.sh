# Cross-item prefetch with extra head rows in AGPRs (RQHIP_CIP="rows,batch,gap,agpr_rows"), K=1024 encode,
# 400 launches per setting, two interleaved passes, experiments library (parity spot check per run).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cipa}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for c in ${CIPS:-64,8,24,0 64,8,24,32 64,8,24,64 64,8,24,96}; do
  echo "== $r $c" >> $O/col.log
  RQHIP_CIP=$c timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 400 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|mismatch|encode" $O/col.log | grep -v "\[\] 0"
echo DONE
