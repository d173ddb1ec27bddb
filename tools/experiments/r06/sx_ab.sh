# Precomputed-syndrome A/B on the release library (rq_debug_apply_sx 1 / 0, one process per setting, two
# interleaved passes; SETTINGS: space-separated settings of +-separated VAR=VALUE, RQHIP_LIB for the
# experiments library's knobs): decode correctness with poisoned erased rows, decode_ms, per-kernel times.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sx}
mkdir -p $O
for r in 1 2; do
for c in ${SETTINGS:-RQ_SX=1 RQ_SX=0}; do
  echo "== $r $c" | tee -a $O/ab.log
  ( export ${c//+/ }; timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${r}_${c//[=,+.\/]/_} -o run -- python3 -u tools/experiments/r06/solve_ab.py ${REPS:-10} >> $O/ab.log 2>&1 ) || { tail -5 $O/ab.log; exit 1; }
  tail -2 $O/ab.log
  f=$(find $O/p_${r}_${c//[=,+.\/]/_} -name "*kernel_stats.csv" | head -1)
  grep -E "k_solve|apply_gi" $f | cut -d, -f1-5
done
done
echo DONE
