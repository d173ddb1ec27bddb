# HBM traffic of the encode column program (rocprofv3 PMC, one counter group per pass, as
# MI355X_MICROARCH.md prescribes): FETCH_SIZE and WRITE_SIZE of the bench workload's encode launch
# and of a same-pattern copy launch of known byte count (calibration).  Then summarise into
# profiles/<tag>_traffic.json (tools/prof_summary.py traffic).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out/pmc_traffic
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/pmc_traffic/fetch -o fetch -- python3 tools/pmc_workload.py > gpurun_out/pmc_traffic/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex rq_colprog --output-format csv -d gpurun_out/pmc_traffic/write -o write -- python3 tools/pmc_workload.py > gpurun_out/pmc_traffic/write.log 2>&1 && \
python3 tools/prof_summary.py traffic gpurun_out/pmc_traffic $TAG > gpurun_out/pmc_traffic/summary.json && \
python3 tools/prof_summary.py traffic gpurun_out/pmc_traffic $TAG rq_colprog_K256_n26 > gpurun_out/pmc_traffic/summary_k256.json
echo EXIT $?
