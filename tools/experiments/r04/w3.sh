# r04: a 3-waves-per-SIMD allocation tier (RQHIP_W3=1: 78 VGPR / 86 AGPR / 52 LDS slots) for the programs
# that fit two waves per SIMD (config 2, K=256): interleaved colbench and bench --config 2 runs, parity
# spot checks by colbench (experiments library).
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04n}
C='col:256,1200,282,1024,20'
B='bench:--config 2 --cpu-sample 0'
run() { local tag=$1; shift; env "$@" bash tools/experiments/run.sh $T/$tag "$C" | sed "s/^/$tag: /"; grep -h mismatching gpurun_out/$T/$tag/1.col.log | sed "s/^/$tag: /"; }
run base1 RQHIP_W3=0 && run w3_1 RQHIP_W3=1 && run base2 RQHIP_W3=0 && run w3_2 RQHIP_W3=1 && \
RQHIP_W3=0 bash tools/experiments/run.sh $T/b_base "$B" > /dev/null && RQHIP_W3=1 bash tools/experiments/run.sh $T/b_w3 "$B" > /dev/null && \
RQHIP_W3=0 bash tools/experiments/run.sh $T/b_base2 "$B" > /dev/null && RQHIP_W3=1 bash tools/experiments/run.sh $T/b_w3_2 "$B" > /dev/null && \
for t in b_base b_w3 b_base2 b_w3_2; do python3 -c "
import json; d=json.load(open('gpurun_out/$T/$t/1.bench.json')); print('$t', d['value'], d['roofline']['launch_ms'])"; done
