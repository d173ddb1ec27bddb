cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -v --timeout 120 --timeout-method thread > $O/test_apply.log 2>&1 || exit $?
for sh in 16,6,2 8,5,2 8,4,2 8,4,1 8,5,1; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$sh -o run -- python -u tools/experiments/r05/apply_ab.py 3 > $O/ab_$sh.log 2>&1 || exit $?
done
