# r02n: Horner passes woven into the next group's production (RQHIP_WEAVE=1) vs run after it, by
# pass count, with cached source loads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02n
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP RQHIP_POLICY=";nt;;sc1" "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h -e encode -e mismatching $O/$n.log | tr '\n' ' ')"
}
for P in 2 3 4 6; do run p$P RQHIP_PASSES=$P; run weave_p$P RQHIP_PASSES=$P RQHIP_WEAVE=1; done
echo DONE
