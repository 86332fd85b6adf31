# gpurun driver (scratch): NS=3 tile study, PMC passes, other-model benches
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/conv_bench.py --batch 1024 --tiles 6,7,11 > gpurun_out/cb_tiles.log 2>&1 || exit 1
bash scripts/pmc_passes.sh gpurun_out/pmc_v12.md --steps 3 --warmup 2 > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 1; }
timeout -k 10 200 python bench.py --arch resnet18 --image-size 448 --batch-size 128 > gpurun_out/bench_r18.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --arch resnet152 --batch-size 256 > gpurun_out/bench_r152.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r18.log | cut -c1-150; tail -1 gpurun_out/bench_r152.log | cut -c1-150
