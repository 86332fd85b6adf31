# side-stream operand protection: record_stream (default) vs hold-until-join, reserved HBM and img/s
cd $GRAFT_REPO_ROOT
L=gpurun_out/protect.log
: > $L
run() { echo "== $1" >> $L; env $2 timeout -k 10 180 python bench.py --steps 30 --warmup 5 2>>gpurun_out/protect_err.log | grep -o '"value": [0-9.]*\|"per_gpu_batch": [0-9]*\|"peak_hbm_gib": [0-9.]*\|"reserved_hbm_gib": [0-9.]*\|"alloc_retries": [0-9]*' | tr '\n' ' ' >> $L; echo >> $L; }
run record "X=0" &&
run keep "IMAGENT_PROTECT=keep" &&
run keep_inflight1 "IMAGENT_PROTECT=keep IMAGENT_MAX_INFLIGHT=1" &&
run keep_cap12 "IMAGENT_PROTECT=keep IMAGENT_MEM_FRACTION=0.12 " &&
run keep_512 "IMAGENT_PROTECT=keep IMAGENT_MEM_FRACTION=0.25"
