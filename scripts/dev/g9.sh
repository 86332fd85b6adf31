set -o pipefail
mkdir -p gpurun_out
IMAGENT_WGRAD_BR=32 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad or conv_fwd_dgrad or stem" --timeout 120 --timeout-method thread > gpurun_out/t9.log 2>&1 && \
IMAGENT_WGRAD_BR=32 timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 > gpurun_out/c9.log 2>&1 && \
IMAGENT_WGRAD_BR=32 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b9_32.log 2>&1 && \
IMAGENT_WGRAD_BR=64 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b9_64.log 2>&1
echo EXIT $?
