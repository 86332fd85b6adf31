set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --tiles 20,21,22 > gpurun_out/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b5.log 2>&1 && \
IMAGENT_CONV_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b5_nostream.log 2>&1
echo EXIT $?
