set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_stream_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t12.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --only 3,224,64,7,2 > gpurun_out/c12.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b12.log 2>&1
echo EXIT $?
