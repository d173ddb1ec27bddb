cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gi2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -v --timeout 120 --timeout-method thread > $O/test_apply.log 2>&1
rc=$?
echo "pytest rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python -u tools/experiments/r05/apply_ab.py 4 > $O/ab.log 2>&1 || exit $?
for sh in 16,6,2 8,6,2 8,5,2 16,5,2 8,6,3 16,6,1 16,6,3 16,4,2 8,4,2; do
  echo "shape $sh" >> $O/sweep.log
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_APPLY_GI=$sh timeout -k 10 120 python -u tools/experiments/r05/apply_ab.py 4 >> $O/sweep.log 2>&1 || exit $?
done
