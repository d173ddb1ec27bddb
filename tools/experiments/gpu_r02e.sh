# r02e: full GPU test suite, then per-object latency (raptorq_eval clone) and fecquic loopback rates.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02e
B=rl-quic-raptor_amd/build
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02e/pytest_gpu.log 2>&1 && \
timeout -k 10 300 $B/raptorq_eval -exp B -schemes raptorq,raptorq-batch -N 32 -K 26 -L 1500 -objMB 3 -trials 5 -p 0,0.05 -seed 1337 -csv gpurun_out/r02e/eval.csv > gpurun_out/r02e/eval_k26.txt 2>&1 && \
timeout -k 10 300 $B/raptorq_eval -exp B -schemes raptorq,raptorq-batch -N 80 -K 64 -L 1200 -objMB 3 -trials 5 -p 0,0.10 -seed 1337 -csv gpurun_out/r02e/eval.csv > gpurun_out/r02e/eval_k64.txt 2>&1 && \
timeout -k 10 300 $B/raptorq_eval -exp B -schemes raptorq,raptorq-batch -N 1100 -K 1024 -L 1200 -objMB 24 -trials 3 -p 0.05 -seed 1337 -csv gpurun_out/r02e/eval.csv > gpurun_out/r02e/eval_k1024.txt 2>&1 && \
head -c 268435456 /dev/urandom > /tmp/fq_in.bin && \
timeout -k 10 200 $B/fecquic loopback --file /tmp/fq_in.bin --out /tmp/fq_out.bin --K 1024 --N 1100 --L 1200 --drop 0.05 --ready held --window 256 --max-blocks 256 --budget 2000000000 > gpurun_out/r02e/fq_k1024_inproc.json 2>&1 && \
timeout -k 10 200 $B/fecquic loopback --file /tmp/fq_in.bin --out /tmp/fq_out2.bin --K 26 --N 32 --L 1200 --drop 0.03 --ready held --window 1024 --max-blocks 4096 --budget 2000000000 > gpurun_out/r02e/fq_k26_inproc.json 2>&1 && \
timeout -k 10 200 $B/fecquic loopback --file /tmp/fq_in.bin --out /tmp/fq_out3.bin --K 128 --N 148 --L 1200 --drop 0.05 --ready held --window 512 --max-blocks 1024 --budget 2000000000 --transport udp > gpurun_out/r02e/fq_k128_udp.json 2>&1
echo EXIT $?
