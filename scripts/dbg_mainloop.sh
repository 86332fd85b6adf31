set -e
for sh in 256,14,256,3,1 2048,7,512,1,1 128,28,128,3,1; do
 for d in 0 1 2 3; do
  echo "== $sh DBG=$d"
  IMAGENT_IGEMM_DBG=$d timeout -k 10 120 python scripts/conv_bench.py --batch 1024 --only $sh --tiles 8,2 2>&1 | grep "tile"
 done
done
