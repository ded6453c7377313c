set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tr}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $OUT/trace.log 2>&1
