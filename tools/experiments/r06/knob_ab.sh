# Allocation-knob sweep with the cross-item prefetch on (ENVS="VAR=val ..."; "-" = defaults), K=1024 encode,
# 400 launches per setting, two interleaved passes, experiments library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-knob}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for c in $ENVS; do
  echo "== $r $c" >> $O/col.log
  ( [ "$c" != "-" ] && export $c; timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 400 >> $O/col.log 2>&1 ) || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $(NF-4)}'
echo DONE
