# r02bd: HBM channel camping check -- the K=1024 encode with the source block stride padded
# (RQBENCH_PAD bytes; blocks are 1 228 800 B = 75 x 16 KiB apart unpadded), release library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02bd
mkdir -p $O
for rep in 1 2; do
  for P in 0 256 4096 1152 65536; do
    env RQBENCH_PAD=$P timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 > $O/pad${P}_$rep.log 2>&1 || exit 1
    echo "pad$P $(grep -h -e encode -e mismatching $O/pad${P}_$rep.log | tr '\n' ' ')"
  done
done
echo DONE
