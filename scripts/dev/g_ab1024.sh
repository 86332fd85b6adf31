# A/B of the existing tuning knobs at the default per-GPU batch 1024 (one MI355X)
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { echo "== $1" >> gpurun_out/ab1024.log; env $2 timeout -k 10 180 python bench.py --steps 30 --warmup 5 2>/dev/null | grep '^{' | cut -c1-200 >> gpurun_out/ab1024.log; }
: > gpurun_out/ab1024.log
run default "X=0" &&
run bnb_all "IMAGENT_STREAM_BNB=all" &&
run bnb_64 "IMAGENT_STREAM_BNB=64" &&
run wgrad_br64 "IMAGENT_WGRAD_BR=64" &&
run wgrad_br32 "IMAGENT_WGRAD_BR=32" &&
run default2 "X=0"
