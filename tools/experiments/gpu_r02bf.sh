# r02bf: does the column program run faster when its source rows are cache-resident?  One round of
# items (B=160: 750 waves, B=192: 900 waves; 196 / 236 MB of source, warm in the 256 MiB Infinity
# Cache across back-to-back launches) against a round of the 1024-block batch (0.48 ms / 5 rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02bf
mkdir -p $O
for rep in 1 2; do
  for B in 160 192 96 1024; do
    timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 $B 30 > $O/b${B}_$rep.log 2>&1 || exit 1
    echo "b$B $(grep -h encode $O/b${B}_$rep.log)"
  done
done
echo DONE
