# r02l: memory-only time of the encode program (RQHIP_DIAG=32 drops the XOR/xtime work) beside the
# full program and the VALU-only floor (RQHIP_DIAG=7).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
run base
run memonly RQHIP_DIAG=32
run memonly_noscr RQHIP_DIAG=33
run memonly_srconly RQHIP_DIAG=43
run valuonly RQHIP_DIAG=7
run memonly_xcd0 RQHIP_DIAG=32 RQHIP_XCD=0
run base_xcd0 RQHIP_XCD=0
run memonly_srccached RQHIP_DIAG=32 RQHIP_POLICY=";nt;;sc1"
run base_srccached RQHIP_POLICY=";nt;;sc1"
echo DONE
