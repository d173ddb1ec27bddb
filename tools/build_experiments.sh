# Builds the experiments variant of librqhip.so (RQHIP_* knobs honoured) into rl-quic-raptor_amd/build_exp/
# for tuning sweeps: RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so python tools/colbench.py ...
# (its own objects and link target: the release library is untouched)
set -e
cd "$(dirname "$0")/../rl-quic-raptor_amd"
make -s -j8 EXPERIMENTS=1 OBJDIR=build_exp/obj build_exp/librqhip.so >/dev/null
