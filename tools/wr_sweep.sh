# word-region kernel timings (bf16 + fp32, B=64) for a few backward grid sizes
set -e
for nb in 256 512; do
  echo "blocks=$nb"; TGFR_BWD_BLOCKS=$nb timeout -k 10 100 python tools/microbench.py 2>&1 | grep "B=64"
done
