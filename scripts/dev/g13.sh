set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t13.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b13.log 2>&1 && \
IMAGENT_STEM_FUSE=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b13_nofuse.log 2>&1
echo EXIT $?
