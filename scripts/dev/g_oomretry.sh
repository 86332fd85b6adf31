# bench.py OOM retry: cap HBM to 12 % (~34 GB) so the 1024 batch cannot fit, expect a retry at 512; then a plain run
set -o pipefail
cd $GRAFT_REPO_ROOT
IMAGENT_MEM_FRACTION=0.12 timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/oom_retry.log 2>&1 &&
timeout -k 10 240 python bench.py > gpurun_out/bench_final.log 2>&1
