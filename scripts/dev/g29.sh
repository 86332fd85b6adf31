set -o pipefail
mkdir -p gpurun_out/p29
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 > gpurun_out/p29/base_$i.log 2>&1 || exit 1
  echo "base $i: $(grep -o '"value": [0-9.]*' gpurun_out/p29/base_$i.log)"
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --main-prio -1 > gpurun_out/p29/prio_$i.log 2>&1 || exit 1
  echo "prio $i: $(grep -o '"value": [0-9.]*' gpurun_out/p29/prio_$i.log)"
done
