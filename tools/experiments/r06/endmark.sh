# (round 6 record: the RQHIP_END_MARKER knob this script A/Bs was removed after it measured no gain, profiles/r06_gap)
# The decode call's marker bound to the apply's dispatch: GPU decode tests, then bench.py A/B
# (experiments library, RQHIP_END_MARKER=1 keeps the separate marker) and a kernel trace of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-endmark}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_apply.py tests/test_gpu_decode_limits.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST FAILED; grep -E "FAILED|Error" $O/pytest.log | tail -20; exit 1; }
tail -1 $O/pytest.log
SETTINGS="RQHIP_END_MARKER=0 RQHIP_END_MARKER=1" bash tools/experiments/r06/sx_bench.sh ${1:-endmark}/ab || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --cpu-sample 0 > $O/prof_bench.json 2> $O/prof.err || exit 1
echo DONE
