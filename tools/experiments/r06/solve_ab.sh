# First-solver A/B (experiments library knobs, one process per setting, two interleaved passes): decode
# correctness with poisoned erased rows, decode_ms, and the kernel trace's per-kernel times.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-solve}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for c in ${SETTINGS:-RQHIP_SOLVE_RR=0 RQHIP_SOLVE_RR=1}; do
  echo "== $r $c" | tee -a $O/ab.log
  ( export $c; timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${r}_${c//[=,]/_} -o run -- python3 -u tools/experiments/r06/solve_ab.py 10 >> $O/ab.log 2>&1 ) || { tail -5 $O/ab.log; exit 1; }
  tail -2 $O/ab.log
  f=$(find $O/p_${r}_${c//[=,]/_} -name "*kernel_stats.csv" | head -1)
  grep -E "k_solve|apply_gi" $f | cut -d, -f1-5
done
done
echo DONE
