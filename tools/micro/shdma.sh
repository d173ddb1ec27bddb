# Row-shared LDS-DMA micro (tools/micro/shdma_gen.py): interleaved rounds of the baseline and shared kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-shdma}
mkdir -p $O
python3 tools/micro/shdma_gen.py /tmp/shdma > $O/gen.log 2>&1 || { tail -5 $O/gen.log; exit 1; }
B="k_base_d16 k_base_d32 k_base_d16_m k_base_d16_v"
S="k_sh_p24_g8 k_sh_p24_g8_m k_sh_p32_g16 k_sh_p32_g16_m k_sh_p48_g16 k_sh_p48_g16_m k_sh_p32_g32 k_sh_p32_g32_m k_sh_p48_g16_v"
for r in 1 2 3; do
  GRID=1024 WGS=64 REPS=40 WARM=20 timeout -k 10 60 tools/micro/shdma_run /tmp/shdma/shdma_base.hsaco $B >> $O/run.log 2>&1 || { echo BASE rc $?; tail -5 $O/run.log; exit 1; }
  GRID=256 WGS=256 REPS=40 WARM=20 timeout -k 10 60 tools/micro/shdma_run /tmp/shdma/shdma_sh.hsaco $S >> $O/run.log 2>&1 || { echo SH rc $?; tail -5 $O/run.log; exit 1; }
done
cat $O/run.log
echo DONE
