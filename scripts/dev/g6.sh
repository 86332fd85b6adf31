set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_stream_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t6.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b6.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_b -o b -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_b.log 2>&1
echo EXIT $?
