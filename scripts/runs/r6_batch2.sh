#!/bin/bash
# round 6, second batch: loader at 448^2 (448 / 320 / 288 stored), bench 2048 vs 4096 with the new BN-apply
# defaults, R50 at 256 img/GPU (bench + per-stream kernel tables), PMC counter calibration on known-byte kernels.
set -o pipefail
O=${1:-gpurun_out/r6b2}
R=$(pwd)
mkdir -p $O
timeout -k 10 600 python -u scripts/loader_bench.py --sizes 448,448@320,448@288 --ranks 8 --threads 2 --dir /tmp/imrec --out $O/loader.md > $O/loader.log 2>&1 || exit 1
for b in 2048 4096 2048 4096; do
  timeout -k 10 300 python -u bench.py --batch-size $b > $O/bench_$b.log 2>&1 || exit 1
  echo "b=$b $(grep '"metric"' $O/bench_$b.log | cut -c1-120) peak $(grep -o '"peak_hbm_gib": [0-9.]*' $O/bench_$b.log)" >> $O/bench_summary.log
done
timeout -k 10 300 python -u bench.py --batch-size 256 --steps 30 > $O/bench_256.log 2>&1 || exit 1
echo "b=256 $(grep '"metric"' $O/bench_256.log | cut -c1-120)" >> $O/bench_summary.log
bash scripts/runs/stream_tables.sh r6b2/st256 --batch-size 256 --steps 10 --warmup 3 || exit 1
hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/hbm_roof.hip -o /tmp/hbm_roof > $O/hbm_build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/cal_f -o f --output-format csv -- /tmp/hbm_roof 1 cal > $R/$O/cal_f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/cal_w -o w --output-format csv -- /tmp/hbm_roof 1 cal > $R/$O/cal_w.log 2>&1 || exit 1
