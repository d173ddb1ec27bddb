cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi10
mkdir -p $O
for sh in 8,4,1,1 8,4,2,1 8,5,1,1 8,5,2,1; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$sh -o run -- python -u tools/experiments/r05/apply_ab.py 2 > $O/ab_$sh.log 2>&1 || exit $?
done
