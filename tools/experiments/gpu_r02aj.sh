# r02aj: source-load cache policy of the column program, A/B interleaved on one box (RQHIP_POLICY =
# "src;out;scratch store;scratch load"; shipped default "nt;nt;;sc1"), encode K=1024 and K=256.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02aj
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, K, N, env...
  local n=$1 K=$2 N=$3; shift 3
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py $K 1200 $N 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h -e encode -e mismatching $O/$n.log | tr '\n' ' ')"
}
for rep in 1 2; do
  for POL in "nt;nt;;sc1" ";nt;;sc1" "sc1;nt;;sc1" ";nt;sc1;sc1" "sc1;nt;sc1;sc1" ";;;sc1"; do
    n=$(echo "k1024_${rep}_$POL" | tr ' ;' '_-')
    run $n 1024 1100 RQHIP_POLICY="$POL"
  done
done
for POL in "nt;nt;;sc1" ";nt;;sc1" "sc1;nt;;sc1"; do
  n=$(echo "k256_$POL" | tr ' ;' '_-')
  run $n 256 282 RQHIP_POLICY="$POL"
done

# k_apply with 4-output-group trimming (release library): kernel stats of the bench
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || exit 1
cat $O/prof_bench.json
find $O/prof -name '*kernel_stats.csv' -exec cut -c1-160 {} \; | head -8
echo DONE
