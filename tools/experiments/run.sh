#!/bin/bash
# One parameterised GPU experiment driver (tools/experiments/README.md): run.sh TAG [STEP ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
BENCH=bench.py
if [ "${LIB:-}" = exp ]; then export RQHIP_LIB=rl-quic-raptor_amd/build_exp/librqhip.so; BENCH=tools/experiments/bench_exp.py; fi
n=0
for step in "$@"; do
  n=$((n + 1)); name=${step%%:*}; arg=""; [ "$step" != "$name" ] && arg=${step#*:}
  log=$O/$n.$name
  case $name in
    tests) timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $log.log 2>&1 \
             || { echo "tests FAILED"; tail -30 $log.log; exit 1; }; tail -1 $log.log ;;
    smoke) timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $log.log 2>&1 || { tail -20 $log.log; exit 1; }; echo smoke ok ;;
    bench) timeout -k 10 300 python3 $BENCH $arg > $log.json 2> $log.err || { tail -20 $log.err; exit 1; }; cat $log.json ;;
    prof) timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $log -o b -- python3 $BENCH --cpu-sample 0 $arg \
             > $log.json 2> $log.err || { echo "prof rc $?"; tail -5 $log.err; exit 1; }
          cp $log/b_kernel_stats.csv $O/kernel_stats_$n.csv 2>/dev/null || find $log -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$n.csv \;
          head -6 $O/kernel_stats_$n.csv | cut -d, -f1-4 ;;
    col) timeout -k 10 150 python3 tools/colbench.py ${arg//,/ } > $log.log 2>&1 || { tail -10 $log.log; exit 1; }; grep -h encode $log.log ;;
    traffic) bash tools/gpu_profile.sh $TAG > $log.log 2>&1 || { tail -10 $log.log; exit 1; }; cp gpurun_out/pmc_traffic/summary.json $O/traffic.json; cp gpurun_out/pmc_traffic/summary_k256.json $O/traffic_k256.json; cat $O/traffic.json $O/traffic_k256.json ;;
    sq) timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
          --kernel-include-regex rq_colprog --output-format csv -d $log -o sq -- python3 tools/colbench.py ${arg:-1024 1200 1100 1024 3} > $log.log 2>&1 || { tail -5 $log.log; exit 1; } ;;
    pmc) # SQ/GRBM counters (two passes) of the kernels matching ARG (default k_apply) over a short bench
        for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
                    "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA"; do
          k=$((${k:-0} + 1))
          timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-include-regex "${arg:-k_apply}" --output-format csv -d $log/p$k -o p \
            -- python3 $BENCH --cpu-sample 0 --steps 3 --warmup 1 > $log.p$k.log 2>&1 || { tail -5 $log.p$k.log; exit 1; }
        done
        python3 tools/experiments/pmc_sum.py $log ;;
    bytes) # HBM traffic of the kernels matching ARG (default k_apply) over a short bench: FETCH_SIZE and
        # WRITE_SIZE in separate passes (per-launch sums in KiB; bytes = KiB x 1024 / the calibration
        # ratio of tools/gpu_profile.sh: 0.5 for FETCH_SIZE, 1.0 for WRITE_SIZE on gfx950)
        for c in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "${arg:-k_apply}" --output-format csv -d $log/p$c -o p \
            -- python3 $BENCH --cpu-sample 0 --steps 3 --warmup 1 > $log.$c.log 2>&1 || { tail -5 $log.$c.log; exit 1; }
        done
        python3 tools/experiments/pmc_sum.py $log ;;
    py) s=${arg%%:*}; a=""; [ "$arg" != "$s" ] && a=${arg#*:}
        timeout -k 10 300 python3 $s $a > $log.log 2>&1 || { tail -20 $log.log; exit 1; }; tail -5 $log.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo DONE
