# Source-load cache policy in the real program (experiments build, RQHIP_POLICY="src;out;scr_st;scr_ld")
# and the overlap micro-benchmark's policy / batching variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05g}
mkdir -p $O
python3 tools/micro/overlap_gen.py /tmp/ov > $O/names.txt || exit 1
N=$(cat $O/names.txt)
[ -n "$SKIP_MICRO" ] || timeout -k 10 120 tools/micro/clockrun /tmp/ov/overlap.hsaco $N > $O/micro.log 2>&1 || { cat $O/micro.log; exit 1; }
[ -n "$SKIP_MICRO" ] || cat $O/micro.log
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for pass in 1 2; do
for pol in ";nt;;sc1" "nt;nt;;sc1" "sc1;nt;;sc1" "sc0 sc1;nt;;sc1" "nt sc1;nt;;sc1" "nt sc0;nt;;sc1"; do
  echo "== $pass $pol" >> $O/col.log
  RQHIP_POLICY="$pol" timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 10 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|encode|mismatch" $O/col.log
echo DONE
