cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sip
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_apply.py -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo tests failed; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python -u tools/experiments/r05/apply_ab.py 3 solve > $O/ab.log 2>&1 || exit $?
grep median $O/ab.log
