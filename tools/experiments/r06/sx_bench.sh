# bench.py (config 3) A/B over experiments-library settings (SETTINGS: space-separated settings of
# comma-separated VAR=VALUE; default the precomputed syndromes on / off), three interleaved passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sxb}
mkdir -p $O
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for r in 1 2 3; do
for c in ${SETTINGS:-RQHIP_APPLY_SX=1 RQHIP_APPLY_SX=0}; do
  t=${c//[=,+]/_}
  ( export ${c//+/ }; timeout -k 10 120 python3 -u bench.py --steps ${STEPS:-100} --warmup 10 > $O/bench_${r}_$t.json 2> $O/bench_${r}_$t.err ) || { tail -5 $O/bench_${r}_$t.err; exit 1; }
  python3 - $O/bench_${r}_$t.json "$r $c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
def find(o, k):
    if isinstance(o, dict):
        for kk, v in o.items():
            if kk == k:
                return v
            r = find(v, k)
            if r is not None:
                return r
print(sys.argv[2], d["value"], "ms", d["ms_per_step"], "enc", find(d, "encode_ms"), "dec", find(d, "decode_ms"), "launch", find(d, "launch_ms"))
PY
done
done
echo DONE
