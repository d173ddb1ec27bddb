# Whole-row prefetch micro-benchmark (tools/micro/rowpf_gen.py): plain timing + GRBM clocks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05e}
mkdir -p $O
python3 tools/micro/rowpf_gen.py /tmp/rp > $O/names.txt || exit 1
N=$(cat $O/names.txt)
timeout -k 10 120 tools/micro/clockrun /tmp/rp/rowpf.hsaco $N > $O/plain.log 2>&1 || { cat $O/plain.log; exit 1; }
cat $O/plain.log
timeout -k 10 120 tools/micro/clockrun /tmp/rp/rowpf.hsaco $N > $O/plain2.log 2>&1 || { cat $O/plain2.log; exit 1; }
cat $O/plain2.log
echo DONE
