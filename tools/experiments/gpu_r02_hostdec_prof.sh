# Host-side phase timing of the host-memory decode pipeline (experiments build, RQHIP_HOST_PROF).
set -e
export TMPDIR=/tmp
O=gpurun_out/hostdec9p
mkdir -p $O
for kt in "2048 1200" "512 256"; do
  RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so RQHIP_HOST_PROF=1 timeout -k 10 200 python tools/hostdec_trace.py $kt 5 > $O/prof_${kt// /_}.log 2>&1
done
