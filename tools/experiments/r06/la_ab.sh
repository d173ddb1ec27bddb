# Look-ahead sweep with the cross-item prefetch on (RQHIP_ALLOC="v,a,la_load,la_reload,max_vmem,lds+1"),
# K=1024 encode, 400 launches per setting, two interleaved passes, experiments library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-la}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for c in ${ALLOCS:-0,0,256,0,0,0 0,0,320,0,0,0 0,0,384,0,0,0 0,0,448,0,0,0 0,0,320,0,60,0}; do
  echo "== $r $c" >> $O/col.log
  RQHIP_ALLOC=$c timeout -k 10 200 python3 tools/colbench.py 1024 1200 1100 1024 400 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $(NF-4)}'
echo DONE
