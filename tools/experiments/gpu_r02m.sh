# r02m: cache-policy bits of the encode program's memory instructions (RQHIP_POLICY =
# "src;out;scratch store;scratch load") on the round-2 schedule, and the schedule at the best one.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
run() {  # name, env...
  local n=$1; shift
  env RQHIP_LIB=$EXP "$@" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/$n.log 2>&1 || exit 1
  echo "$n $(grep -h encode $O/$n.log)"
}
run base
for POL in "nt;nt;;sc1" ";nt;;sc1" ";;;sc1" ";nt;;" ";nt;sc1;sc1" ";nt;nt;sc1" ";nt;;sc0" "sc0;nt;;sc1" "sc1;nt;;sc1" ";nt;sc0 sc1;sc0 sc1"; do
  n=$(echo "pol_$POL" | tr ' ;' '_-')
  run $n RQHIP_POLICY="$POL"
done
for P in 1 2 3 4; do run src_cached_p$P RQHIP_POLICY=";nt;;sc1" RQHIP_PASSES=$P; done
echo DONE
