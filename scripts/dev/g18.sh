set -o pipefail
mkdir -p gpurun_out/v6
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v6 -o v6 -- python3 bench.py --steps 6 --warmup 1 > gpurun_out/v6/prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch-size 256 > gpurun_out/v6/b256.log 2>&1 && \
timeout -k 10 300 python -u bench.py --batch-size 1024 > gpurun_out/v6/b1024.log 2>&1 && \
timeout -k 10 300 python -u bench.py --dtype fp8 > gpurun_out/v6/fp8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --dtype fp8 --batch-size 1024 --optimizer lars > gpurun_out/v6/fp8_1024_lars.log 2>&1 && \
timeout -k 10 300 python -u bench.py --arch resnet152 --batch-size 256 > gpurun_out/v6/r152.log 2>&1 && \
timeout -k 10 300 python -u bench.py --arch resnet18 --image-size 448 --batch-size 128 > gpurun_out/v6/r18_448.log 2>&1 && \
timeout -k 10 300 python -u bench.py --kernels torch --batch-size 256 > gpurun_out/v6/torch256.log 2>&1
echo EXIT $?
