# The code warm-up's four loads into an LDS sink without the wait (RQHIP_CODEPF=2) against the shipped
# prefetch-and-wait (1): parity + encode launch (colbench), then the bench, interleaved, experiments library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-codepf}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2 3; do
for m in 1 2; do
  echo "== $r $m" >> $O/col.log
  RQHIP_CODEPF=$m timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 20 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
done
done
for r in 1 2; do
for m in 1 2; do
  RQHIP_CODEPF=$m timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/b${r}_$m.json 2> $O/b${r}_$m.err || { tail -5 $O/b${r}_$m.err; exit 1; }
done
done
grep -E "==|mismatch|encode" $O/col.log
for f in $O/b*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"; done
echo DONE
