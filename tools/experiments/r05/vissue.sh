# VALU issue-rate micro-benchmark (tools/micro/vissue_gen.py): GRBM clock and cycles per kernel at N = 20k
# and 40k instructions per wave (the slope removes the launch overhead)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r05c}
mkdir -p $O
for n in 20000 40000; do
VI_N=$n python3 tools/micro/vissue_gen.py /tmp/vi$n > $O/names.txt || exit 1
N=$(cat $O/names.txt)
GRID=1024 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/pmc$n -o p -- tools/micro/clockrun /tmp/vi$n/vissue.hsaco $N > $O/pmc$n.log 2>&1 || { echo pmc fail; tail -5 $O/pmc$n.log; exit 1; }
python3 tools/micro/pmc_clock.py $O/pmc$n/p_counter_collection.csv $n
done
echo DONE
