set -e
for nb in 256 512 1024; do
  echo "blocks=$nb"; TGFR_BWD_BLOCKS=$nb timeout -k 10 100 python tools/microbench.py 2>&1 | grep "B=64"
done
