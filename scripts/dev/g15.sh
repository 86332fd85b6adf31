set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t15.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b15.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b15b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_b -o b -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_b.log 2>&1
echo EXIT $?
