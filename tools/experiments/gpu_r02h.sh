# r02h: 5-VALU xtime, SALU-free scratch offsets and age-coalesced waits -- GPU parity, then the
# encode launch time vs IR schedule, wait coalescing and 2-wave residency (experiments library).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02h
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
for P in 0 1 2 3 4; do run p$P RQHIP_PASSES=$P; done
for W in 0,0 60,8 320,48 640,96; do run w${W/,/_} RQHIP_WAIT_AGE=$W; done
for P in 1 2 3 4 6; do run two_p$P RQHIP_PASSES=$P RQHIP_ALLOC=116,128,0,0,0,79; done
echo DONE
