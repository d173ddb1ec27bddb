cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -x -q --timeout 120 --timeout-method thread > $O/test_rel.log 2>&1 || { echo rel tests failed; exit 1; }
for sh in 4,4,1,2 12,5,2,1; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -x -q --timeout 120 --timeout-method thread > $O/test_$sh.log 2>&1 || { echo tests $sh failed; exit 1; }
done
for sh in 8,5,2,1 12,5,2,1 12,5,1,1 4,5,1,2 4,4,1,2 8,5,1,2 12,4,2,1; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$sh -o run -- python -u tools/experiments/r05/apply_ab.py 2 > $O/ab_$sh.log 2>&1 || exit $?
done
