#!/bin/bash
# A/B of the v3 256x256-tile K threshold on the full bench step, interleaved in one box
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for rep in 1 2; do
  for k in 0 512 1024 100000; do
    echo "== IMAGENT_V3_256_MINK=$k rep $rep"
    IMAGENT_V3_256_MINK=$k timeout -k 10 200 python bench.py --steps 15 --warmup 4 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
