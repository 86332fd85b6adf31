set -o pipefail
mkdir -p gpurun_out/p30
run() { n=$1; shift; timeout -k 10 240 python3 bench.py "$@" > gpurun_out/p30/$n.log 2>&1 || exit 1; echo "$n: $(grep -o '"value": [0-9.]*, [^}]*ms_per_step": [0-9.]*' gpurun_out/p30/$n.log | sed 's/"unit.*ms_per/ ms_per/')"; }
run r50_b256 --batch-size 256 --steps 10 --warmup 3
run r50_fp8 --dtype fp8 --steps 10 --warmup 5
run r152_b256 --arch resnet152 --batch-size 256 --steps 6 --warmup 3
run r18_448 --arch resnet18 --image-size 448 --batch-size 128 --steps 10 --warmup 3
run r50_graph --graph 1 --steps 10 --warmup 3
