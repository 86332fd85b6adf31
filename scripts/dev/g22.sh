set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_stream_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t22.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --only 256,56,64,1,1 > gpurun_out/c22.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --only 256,56,128,1,1 >> gpurun_out/c22.log 2>&1 && \
IMAGENT_CONV_STREAM=0 timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --only 256,56,128,1,1 >> gpurun_out/c22.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/b22.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/b22b.log 2>&1
echo EXIT $?
