set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_stream_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t19.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --only 64,56,64,3,1 --tiles 1,3,4,5,6 > gpurun_out/c19.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --only 64,56,256,1,1 --tiles 1,3,4,5,6 >> gpurun_out/c19.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/b19.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/b19b.log 2>&1
echo EXIT $?
