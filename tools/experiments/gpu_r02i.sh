# r02i: source loads through the row-offset SGPR window -- GPU parity, then schedule / wait-age sweeps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/release.log 2>&1 || exit 1
grep -h encode $O/release.log
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
for P in 1 2 3 4; do run p$P RQHIP_PASSES=$P; done
for W in 320,48 480,64; do for P in 2 3; do run w${W/,/_}_p$P RQHIP_WAIT_AGE=$W RQHIP_PASSES=$P; done; done
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
echo DONE
