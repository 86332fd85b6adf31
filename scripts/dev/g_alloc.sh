# caching-allocator footprint: plain vs expandable segments, with and without a 12 % HBM cap
cd $GRAFT_REPO_ROOT
L=gpurun_out/alloc.log
: > $L
run() { echo "== $1" >> $L; env $2 timeout -k 10 180 python bench.py --steps 30 --warmup 5 2>>gpurun_out/alloc_err.log | grep -o '"value": [0-9.]*\|"per_gpu_batch": [0-9]*\|"peak_hbm_gib": [0-9.]*\|"reserved_hbm_gib": [0-9.]*\|"alloc_retries": [0-9]*' | tr '\n' ' ' >> $L; echo >> $L; }
run plain "X=0" &&
run expandable "PYTORCH_HIP_ALLOC_CONF=expandable_segments:True" &&
run cap12 "IMAGENT_MEM_FRACTION=0.12" &&
run cap12_expandable "IMAGENT_MEM_FRACTION=0.12 PYTORCH_HIP_ALLOC_CONF=expandable_segments:True"
