# k_solve's grid (the general solver, launched on every async decode, almost never with a block to
# solve): 256 workgroups (shipped) against 64 / 16; kernel trace of the decode A/B script.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gsolve
mkdir -p $O
for r in 1 2; do
for g in 256 64 16; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_GSOLVE_GRID=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p${r}_$g -o run -- python -u tools/experiments/r05/apply_ab.py 2 > $O/ab${r}_$g.log 2>&1 || exit $?
done
done
