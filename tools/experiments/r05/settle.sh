# The bench's 20-step line with and without ~300 ms of untimed steps before its warmup (do the timed steps
# see the GPU's power management ramping up?), interleaved, then a 200-step line.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-settle}
mkdir -p $O
for r in 1 2 3; do
for m in 0 300; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --settle-ms $m > $O/b${r}_$m.json 2> $O/b${r}_$m.err || { tail -5 $O/b${r}_$m.err; exit 1; }
done
done
timeout -k 10 600 python3 -u bench.py --steps 200 --warmup 5 --cpu-sample 0 > $O/b200.json 2> $O/b200.err || exit 1
for f in $O/b*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['launch_ms'], d['config']['settle'])"; done
echo DONE
