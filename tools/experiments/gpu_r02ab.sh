# r02ab: small-K column programs at two or four waves per SIMD (RQHIP_ALLOC caps the registers and
# LDS slots per wave) against one: config 2 (K=256) and colbench at K=128 / 512.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ab
mkdir -p $O
EXP=rl-quic-raptor_amd/build_exp/librqhip.so
for A in "0,0,0,0,0,0" "122,128,0,0,0,79" "58,64,0,0,0,40"; do
  n=$(echo $A | tr ',' '_')
  RQHIP_LIB=$EXP RQHIP_ALLOC=$A timeout -k 10 200 python3 bench.py --config 2 --cpu-sample 0 > $O/cfg2_$n.json 2> $O/cfg2_$n.err || { tail -5 $O/cfg2_$n.err; exit 1; }
  echo "cfg2 $A $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["value"], d["roofline"]["launch_ms"])' $O/cfg2_$n.json)"
  for KN in "128 1200 148" "512 1200 571"; do
    set -- $KN
    RQHIP_LIB=$EXP RQHIP_ALLOC=$A timeout -k 10 120 python3 tools/colbench.py $1 $2 $3 1024 20 > $O/cb_${1}_$n.log 2>&1 || exit 1
    echo "K=$1 $A $(grep -h -e 'encode K' -e mismatching $O/cb_${1}_$n.log | tr '\n' ' ')"
  done
done
echo DONE
