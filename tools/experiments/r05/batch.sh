# Source-load batching in the real program (experiments build, RQHIP_LOAD_BATCH=B): two interleaved passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05k}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for pass in 1 2 3; do
for b in 1 2 4 8; do
  echo "== $pass batch $b" >> $O/col.log
  RQHIP_LOAD_BATCH=$b timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $4, $(NF-4)}'
echo DONE
