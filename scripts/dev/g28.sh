set -o pipefail
mkdir -p gpurun_out/p28
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p28/k1024 -o k -- python3 bench.py --batch-size 1024 --steps 3 --warmup 2 > gpurun_out/p28/k1024.log 2>&1 && \
echo "1024: $(grep metric gpurun_out/p28/k1024.log | cut -c80-140)" && \
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/p28/b512.log 2>&1 && \
echo "512: $(grep metric gpurun_out/p28/b512.log | cut -c80-140)"
