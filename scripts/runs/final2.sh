#!/bin/bash
# end-of-round: the bench table at HEAD, then the per-stream kernel tables of the 4096-img step
set -o pipefail
bash scripts/runs/final_bench.sh gpurun_out/fbench7 || exit 1
bash scripts/runs/stream_tables.sh r6final --steps 4 --warmup 2 || exit 1
