# Packed index dwords (two subset numbers per dword) against the shipped shape: apply parity tests under
# the packed shape, then interleaved rocprof runs of both.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gipack
mkdir -p $O
RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=8,5,2,1,1 timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -x -q --timeout 120 --timeout-method thread > $O/test_pack.log 2>&1 || { echo tests failed; exit 1; }
for r in 1 2; do
for sh in 8,5,2,1,0 8,5,2,1,1 8,5,1,1,1; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p${r}_$sh -o run -- python -u tools/experiments/r05/apply_ab.py 2 > $O/ab${r}_$sh.log 2>&1 || exit $?
done
done
