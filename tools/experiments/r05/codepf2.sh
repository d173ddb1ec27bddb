# Second A/B of RQHIP_CODEPF 2 vs 1 with the order alternated per pass (experiments library).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-codepf2}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2 3 4; do
  if [ $((r % 2)) -eq 0 ]; then ms="2 1"; else ms="1 2"; fi
  for m in $ms; do
    echo "== $r $m" >> $O/col.log
    RQHIP_CODEPF=$m timeout -k 10 120 python3 tools/colbench.py 1024 1200 1100 1024 40 >> $O/col.log 2>&1 || { tail -5 $O/col.log; exit 1; }
  done
done
for r in 1 2 3; do
  if [ $((r % 2)) -eq 0 ]; then ms="2 1"; else ms="1 2"; fi
  for m in $ms; do
    RQHIP_CODEPF=$m timeout -k 10 200 python3 -u bench.py --steps 40 --warmup 5 --cpu-sample 0 > $O/b${r}_$m.json 2> $O/b${r}_$m.err || { tail -5 $O/b${r}_$m.err; exit 1; }
  done
done
grep -E "==|encode" $O/col.log | paste - - | awk '{print $2, $3, $(NF-4)}'
for f in $O/b*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"; done
echo DONE
