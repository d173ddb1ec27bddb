# r04: first runs of the two-wave (pair) column program: a small smoke launch, then encode launch A/B
# (experiments build, RQHIP_PAIR=1 vs 0) at K=1024 (config 3) and K=2048.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04c
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
RQHIP_PAIR=1 timeout -k 10 90 python3 tools/colbench.py 1024 1200 1100 16 3 > gpurun_out/r04c/pair_small.log 2>&1 || { echo SMALL FAILED rc=$?; tail -20 gpurun_out/r04c/pair_small.log; exit 1; }
tail -3 gpurun_out/r04c/pair_small.log
RQHIP_PAIR=1 timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 10 > gpurun_out/r04c/pair.log 2>&1 || { echo PAIR FAILED; tail -20 gpurun_out/r04c/pair.log; exit 1; }
RQHIP_PAIR=0 timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 10 > gpurun_out/r04c/single.log 2>&1 || { echo SINGLE FAILED; tail -20 gpurun_out/r04c/single.log; exit 1; }
RQHIP_PAIR=1 timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 10 > gpurun_out/r04c/pair2.log 2>&1 || exit 1
RQHIP_PAIR=0 timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 10 > gpurun_out/r04c/single2.log 2>&1 || exit 1
RQHIP_PAIR=1 timeout -k 10 120 python3 tools/colbench.py 2048 1200 2260 512 10 > gpurun_out/r04c/pair_k2048.log 2>&1 || exit 1
RQHIP_PAIR=0 timeout -k 10 120 python3 tools/colbench.py 2048 1200 2260 512 10 > gpurun_out/r04c/single_k2048.log 2>&1 || exit 1
grep -h encode gpurun_out/r04c/*.log
