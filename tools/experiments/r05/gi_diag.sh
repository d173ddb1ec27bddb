cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi7
mkdir -p $O
for d in 0 1 2 3 4 6 7; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=8,5,2 RQHIP_APPLY_DIAG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$d -o run -- python -u tools/experiments/r05/apply_ab.py 2 > $O/ab_$d.log 2>&1
done
exit 0
