# run-ahead limit (StepRunner.max_inflight): img/s and reserved HBM for 1, 2, 3 and unlimited in-flight steps
cd $GRAFT_REPO_ROOT
L=gpurun_out/inflight.log
: > $L
run() { echo "== $1" >> $L; env $2 timeout -k 10 180 python bench.py --steps 30 --warmup 5 2>>gpurun_out/inflight_err.log | grep -o '"value": [0-9.]*\|"per_gpu_batch": [0-9]*\|"peak_hbm_gib": [0-9.]*\|"reserved_hbm_gib": [0-9.]*\|"alloc_retries": [0-9]*' | tr '\n' ' ' >> $L; echo >> $L; }
run default2 "X=0" &&
run inflight1 "IMAGENT_MAX_INFLIGHT=1" &&
run inflight3 "IMAGENT_MAX_INFLIGHT=3" &&
run unlimited "IMAGENT_MAX_INFLIGHT=0" &&
run cap12_default2 "IMAGENT_MEM_FRACTION=0.12" &&
run default2_again "X=0"
