set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --main-priority 1 > gpurun_out/b11_p1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --main-priority 0 > gpurun_out/b11_p0.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --main-priority 1 > gpurun_out/b11_p1b.log 2>&1
echo EXIT $?
