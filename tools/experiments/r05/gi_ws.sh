cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi8
mkdir -p $O
for cfg in 8,5,2:1 8,5,2:2 8,5,2:4 8,5,1:4 8,4,1:4; do
  sh=${cfg%:*}; ws=${cfg#*:}
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh RQHIP_APPLY_WS=$ws timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${sh}_$ws -o run -- python -u tools/experiments/r05/apply_ab.py 2 > $O/ab_${sh}_$ws.log 2>&1 || exit $?
done
