# Builds the experiments variant of librqhip.so (RQHIP_* knobs honoured) into rl-quic-raptor_amd/build_exp/
# for tuning sweeps: RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so python tools/colbench.py ...
set -e
cd "$(dirname "$0")/../rl-quic-raptor_amd"
mkdir -p build_exp
make -s -j8 EXPERIMENTS=1 OBJDIR=build_exp/obj build/librqhip.so >/dev/null
cp build/librqhip.so build_exp/librqhip.so
rm -f build/librqhip.so && make -s -j8 OBJDIR=build/obj build/librqhip.so  # relink the release library
