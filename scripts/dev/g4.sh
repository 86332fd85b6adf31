set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_b -o b -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_b.log 2>&1
echo EXIT $?
