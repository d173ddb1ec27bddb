# Config 5 (host-memory stream) with the descriptor fetch (RQHIP_DEC_ZC=3, the default) against the
# side-stream upload (2), interleaved, experiments library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-cfg5d}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
for m in 3 2; do
  RQHIP_DEC_ZC=$m timeout -k 10 300 python3 bench.py --config 5 --cpu-sample 0 > $O/b${r}_$m.json 2> $O/b${r}_$m.err || { tail -5 $O/b${r}_$m.err; exit 1; }
done
done
for f in $O/b*.json; do python3 -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], r['achieved'], r['peak'])"; done
echo DONE
