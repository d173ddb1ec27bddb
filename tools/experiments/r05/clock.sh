set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
python3 tools/micro/clock_gen.py /tmp/clk > $O/names.txt || exit 1
N=$(cat $O/names.txt)
timeout -k 10 120 tools/micro/clockrun /tmp/clk/clock.hsaco $N > $O/clock_plain.log 2>&1 || { cat $O/clock_plain.log; exit 1; }
cat $O/clock_plain.log
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/clk -o clk -- tools/micro/clockrun /tmp/clk/clock.hsaco $N > $O/clock_pmc.log 2>&1 || { echo pmc fail; tail -5 $O/clock_pmc.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex rq_colprog --output-format csv -d $O/col -o col -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/col.log 2>&1 || { echo col fail; tail -5 $O/col.log; exit 1; }
export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so
for d in 4 32; do
RQHIP_DIAG=$d timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex rq_colprog --output-format csv -d $O/col_d$d -o col -- python3 tools/colbench.py 1024 1200 1100 1024 3 > $O/col_d$d.log 2>&1 || { echo col d$d fail; tail -5 $O/col_d$d.log; exit 1; }
done
echo DONE
