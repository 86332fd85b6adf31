set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --no-stats > gpurun_out/c_nostats.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --epi 2 > gpurun_out/c_epi2.log 2>&1 && \
timeout -k 10 200 python -u scripts/conv_bench.py --batch 512 --epi 1 > gpurun_out/c_epi1.log 2>&1 && \
timeout -k 10 300 python -u scripts/conv_bench.py --batch 512 --tiles 2,4,8,9 > gpurun_out/c_tiles.log 2>&1
echo EXIT $?
