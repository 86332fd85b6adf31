set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python bench.py > gpurun_out/bench1024_a.log 2>&1 &&
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/bench1024_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1024 -o run -- python3 bench.py --steps 5 --warmup 3 > gpurun_out/prof1024.log 2>&1
