cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/marks; mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/base_$r.json 2> $O/base_$r.err || exit 1
  RQHIP_NOMARK=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/nomark_$r.json 2> $O/nomark_$r.err || exit 1
done
for f in $O/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['config']['encode_ms'], d['config']['decode_ms'])"; done
RQHIP_NOMARK=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python -u bench.py --steps 10 --warmup 3 > $O/prof.json 2> $O/prof.err || exit 1
