# Encode column-program sweep (K=1024 T=1200 N=1100, 1024 blocks).  Args: ALLOC[:LDS_HORIZON] ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/sweep2.log
for arg in "$@"; do
  o=${arg%%:*}; h=2000; [ "$arg" != "$o" ] && h=${arg#*:}
  echo "== RQHIP_ALLOC=$o RQHIP_LDS_HORIZON=$h" >> gpurun_out/sweep2.log
  RQHIP_ALLOC=$o RQHIP_LDS_HORIZON=$h timeout -k 10 120 python -u tools/colbench.py 1024 1200 1100 1024 10 >> gpurun_out/sweep2.log 2>&1 || exit 3
done
echo EXIT $?
