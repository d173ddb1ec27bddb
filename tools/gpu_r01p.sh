#!/bin/bash
# r01p: host-memory batch API parity + e2e rate, and the VALU-floor sweep over waves per SIMD.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_batch.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r01p_tests.log 2>&1 &&
timeout -k 10 180 python -u tools/e2e_host_api.py 1024 3 > gpurun_out/r01p_e2e_host.json 2> gpurun_out/r01p_e2e_host.err &&
timeout -k 10 600 python tools/sweep.py gpurun_out/sweep10.log '[{"RQHIP_DIAG": "7"}, {"RQHIP_DIAG": "7", "RQHIP_ALLOC": "120,128,0,0,0,79"}, {"RQHIP_DIAG": "7", "RQHIP_ALLOC": "78,80,0,0,0,53"}, {"RQHIP_DIAG": "15"}, {"RQHIP_ALLOC": "120,128,0,0,0,79"}]'
