# Source rows staged in LDS by per-row DMA (buffer_load_dword ... lds, no VGPR held in flight) at
# look-aheads of 600-1000 IR nodes, against register prefetch only (0); experiments library, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ladma}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for pass in 1 2; do
for la in 0 600 800 1000; do
  echo "== $pass $la" >> $O/col.log
  RQHIP_LA_DMA=$la timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
grep -E "==|mismatch|encode" $O/col.log
echo DONE
