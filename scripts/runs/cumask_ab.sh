#!/bin/bash
# A/B: the weight-gradient side stream confined to q/4 of the CUs (IMAGENT_SIDE_CUMASK) at the 4096 default
set -o pipefail
O=${1:-gpurun_out/cumask}
mkdir -p $O
run() { local tag=$1 q=$2; shift 2; IMAGENT_SIDE_CUMASK=$q timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || exit 1; echo "$tag q=$q $(grep -o '"value": [0-9.]*' $O/$tag.log)" >> $O/summary.log; }
run base_a 0 --steps 12 --warmup 4
run q2_a 2 --steps 12 --warmup 4
run q1_a 1 --steps 12 --warmup 4
run q3_a 3 --steps 12 --warmup 4
run base_b 0 --steps 12 --warmup 4
run q2_b 2 --steps 12 --warmup 4
run q3_b 3 --steps 12 --warmup 4
