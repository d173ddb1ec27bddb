# First-round synchronisation: odd workgroups start n x 8128 cycles late (RQHIP_STAGGER, experiments build),
# and the steady-state rate of a 4096-block batch; two interleaved passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05i}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for pass in 1 2; do
for st in 0 1 2 3 5; do
  echo "== $pass stagger $st" >> $O/col.log
  RQHIP_STAGGER=$st timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
echo "== $pass blocks 4096" >> $O/col.log
timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 4096 10 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $4, $(NF-4)}'
echo DONE
