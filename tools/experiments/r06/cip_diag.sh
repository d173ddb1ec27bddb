cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for c in ${CIPS:-0,8,24 64,8,24}; do
  echo "== $c"
  RQHIP_CIP=$c timeout -k 10 200 python3 tools/experiments/r06/cip_diag.py || exit 1
done
echo "== release"
unset RQHIP_LIB
timeout -k 10 200 python3 tools/experiments/r06/cip_diag.py || exit 1
echo DONE
