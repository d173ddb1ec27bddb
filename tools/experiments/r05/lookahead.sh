# Source-load policy x look-ahead / outstanding-load budget in the real program (experiments build):
# RQHIP_POLICY="src;out;scr_st;scr_ld", RQHIP_ALLOC="v,a,la_load,la_reload,max_vmem,lds+1"; two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05j}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for pass in 1 2; do
for pol in ";nt;;sc1" "nt;nt;;sc1"; do
for al in "0,0,0,0,0,0" "0,0,480,0,60,0" "0,0,640,0,60,0" "0,0,960,0,60,0" "0,0,240,0,0,0"; do
  echo "== $pass $pol $al" >> $O/col.log
  RQHIP_POLICY="$pol" RQHIP_ALLOC="$al" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $4, $(NF-4)}'
echo DONE
