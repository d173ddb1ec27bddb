# Memory/VALU overlap micro-benchmark (tools/micro/overlap_gen.py), two interleaved passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05f}
mkdir -p $O
python3 tools/micro/overlap_gen.py /tmp/ov > $O/names.txt || exit 1
N=$(cat $O/names.txt)
for p in 1 2; do
timeout -k 10 120 tools/micro/clockrun /tmp/ov/overlap.hsaco $N > $O/plain$p.log 2>&1 || { cat $O/plain$p.log; exit 1; }
cat $O/plain$p.log
GRID=1280 WGS=256 timeout -k 10 60 tools/micro/clockrun /tmp/ov/overlap_wg4.hsaco k_wg4_d16 > $O/wg4_$p.log 2>&1 || { cat $O/wg4_$p.log; exit 1; }
cat $O/wg4_$p.log
done
echo DONE
