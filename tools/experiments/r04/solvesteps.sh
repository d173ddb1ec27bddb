# r04: where k_solve_pq<1,4>'s 64 us go: the first pass limited to N pivot steps (RQHIP_SOLVE_STEPS, timing
# only: X is wrong, so the bench runs without its checks), kernel stats of each (experiments library).
cd $GRAFT_REPO_ROOT
export LIB=exp
T=${1:-r04k}
for n in 1 13 26 39; do
  RQHIP_SOLVE_STEPS=$n bash tools/experiments/run.sh $T/s$n "prof:--no-verify" > /dev/null || exit 1
  echo "steps $n: $(grep -h k_solve_pq gpurun_out/$T/s$n/kernel_stats_1.csv | cut -d, -f1-4)"
done
bash tools/experiments/run.sh $T/sall "prof" > /dev/null && echo "all: $(grep -h k_solve_pq gpurun_out/$T/sall/kernel_stats_1.csv | cut -d, -f1-4)"
