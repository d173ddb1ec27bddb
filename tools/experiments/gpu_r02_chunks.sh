# Host-memory pipeline chunk sizing sweep (experiments build): RQHIP_CHUNKS x RQHIP_CHUNK_MIB.
set -e
export TMPDIR=/tmp
O=gpurun_out/chunks
mkdir -p $O
for cfg in "8 16" "4 32" "6 24" "3 48"; do
  set -- $cfg
  for kt in "512 256" "128 1200" "2048 1200"; do
    echo "chunks=$1 mib=$2 K,T=$kt" >> $O/sweep.log
    RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_CHUNKS=$1 RQHIP_CHUNK_MIB=$2 timeout -k 10 200 python tools/hostdec_trace.py $kt 5 2>&1 | grep decode | tail -3 >> $O/sweep.log
  done
done
