# First-solver A/B between two builds of the experiments library (LIBS="a.so b.so"), one process each,
# two interleaved passes: decode correctness with poisoned erased rows, decode_ms, kernel-trace times.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-solvelib}
mkdir -p $O
for r in 1 2; do
for L in ${LIBS:-rl-quic-raptor_amd/build_exp_old/librqhip.so rl-quic-raptor_amd/build_exp/librqhip.so}; do
  t=$(echo $L | cut -d/ -f2)
  echo "== $r $t" >> $O/ab.log
  ( export RQHIP_LIB=$L; timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${r}_$t -o run -- python3 -u tools/experiments/r06/solve_ab.py 10 >> $O/ab.log 2>&1 ) || { tail -5 $O/ab.log; exit 1; }
done
done
python3 - $O <<'PY'
import csv, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/p_*/run_kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "solve" in r["Name"] or "apply_gi" in r["Name"]:
            print(f.split("/")[-2], r["Name"][:34], r["AverageNs"], r["MinNs"])
PY
grep -E "==|solved|decode_ms" $O/ab.log
echo DONE
