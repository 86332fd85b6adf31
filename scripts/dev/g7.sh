set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad or conv_fwd_dgrad or stem" --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 > gpurun_out/c7.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b7.log 2>&1
echo EXIT $?
