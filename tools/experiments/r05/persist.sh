# Overlap micro-benchmark, persistent variants (grid 1024, 5 items per wave) beside the one-item-per-wave ones
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05h}
mkdir -p $O
python3 tools/micro/overlap_gen.py /tmp/ov > /dev/null || exit 1
for p in 1 2; do
timeout -k 10 60 tools/micro/clockrun /tmp/ov/overlap.hsaco k_d16_v20 k_nt_d16 k_ntsc1_d16 k_batch4_d16 > $O/g5120_$p.log 2>&1 || { cat $O/g5120_$p.log; exit 1; }
cat $O/g5120_$p.log
GRID=1024 timeout -k 10 60 tools/micro/clockrun /tmp/ov/overlap_p.hsaco k_p_d16 k_p_nt_d16 k_p_ntsc1_d16 k_p_batch4_d16 k_p_d32 k_p_nt_d32 > $O/p_$p.log 2>&1 || { cat $O/p_$p.log; exit 1; }
cat $O/p_$p.log
done
echo DONE
