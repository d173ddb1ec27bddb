# r02q: per-object API latency (tools/perobj_latency.py) and the raptorq_eval clone at the
# reference's exp B shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 300 python3 tools/perobj_latency.py 50 > $O/perobj_latency.json 2> $O/perobj.err || { tail -20 $O/perobj.err; exit 1; }
cat $O/perobj_latency.json
E=rl-quic-raptor_amd/build/raptorq_eval
timeout -k 10 200 $E -exp B -schemes raptorq,raptorq-batch -N 80 -K 64 -L 1200 -objMB 3 -trials 20 -p 0.1 -seed 1337 > $O/eval_k64.log 2>&1 || exit 1
timeout -k 10 200 $E -exp B -schemes raptorq,raptorq-batch -N 282 -K 256 -L 1200 -objMB 3 -trials 20 -p 0.05 -seed 1337 > $O/eval_k256.log 2>&1 || exit 1
timeout -k 10 200 $E -exp B -schemes raptorq,raptorq-batch -N 1100 -K 1024 -L 1200 -objMB 6 -trials 10 -p 0.05 -seed 1337 > $O/eval_k1024.log 2>&1 || exit 1
timeout -k 10 200 $E -exp B -schemes raptorq,raptorq-batch -N 32 -K 26 -L 1500 -objMB 3 -trials 20 -p 0.1 -seed 1337 > $O/eval_k26.log 2>&1 || exit 1
grep -h "scheme=" $O/eval_*.log
echo DONE
