# The apply's recovered-row store policy (RQHIP_APPLY_STPOL: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1; experiments
# library): does the ~5 us between the apply and the next encode come from dirty lines at its end?
# Bench kernel traces, two passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-stpol}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for p in 0 1 2 3; do
  RQHIP_APPLY_STPOL=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p${r}_$p -o run -- python3 -u bench.py --steps 12 --warmup 3 --cpu-sample 0 > $O/b${r}_$p.json 2> $O/b${r}_$p.err || { tail -5 $O/b${r}_$p.err; exit 1; }
done
done
echo DONE
