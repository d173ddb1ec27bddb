# The column program's full / memory-only (RQHIP_DIAG=4) / no-load (32) builds timed over 400 launches
# (the clocks settle within the first ~100), experiments library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cap}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for d in 0 4 32; do
  echo "== $r $d" >> $O/col.log
  RQHIP_DIAG=$d timeout -k 10 200 python3 tools/colbench.py 1024 1200 1100 1024 400 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $(NF-4)}'
echo DONE
