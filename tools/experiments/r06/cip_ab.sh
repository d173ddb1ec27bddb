# Cross-item prefetch A/B (AllocOpts::cip, RQHIP_CIP="rows,batch,gap"): the K=1024 encode launch over 400
# launches per setting (clocks settle within ~100), two interleaved passes, experiments library; each run
# spot-checks two blocks against the oracle first.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cip}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for c in 0,8,24 32,8,24 64,8,24 64,16,48 96,8,24; do
  echo "== $r $c" >> $O/col.log
  RQHIP_CIP=$c timeout -k 10 200 python3 tools/colbench.py 1024 1200 1100 1024 400 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|mismatch|encode" $O/col.log
echo DONE
