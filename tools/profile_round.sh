#!/bin/bash
# Collect the round's rocprofv3 evidence on a GPU box (run from the repo root):
#   1. kernel trace + stats of the bench command (graph replay)
#   2. FETCH_SIZE and 3. WRITE_SIZE PMC passes (separate runs: TCC slot
#      limits), eager launches, few steps.
# Then, here: python tools/summarize_profile.py gpurun_out/prof_<tag> profiles/<round> <config_key>
# Usage: bash tools/profile_round.sh <tag> [extra bench.py args...]
#   e.g. bash tools/profile_round.sh r02_cfg2
#        bash tools/profile_round.sh r02_cfg5 --batch 128 --words 64 --precision fp32
set -e
TAG=${1:-r02}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" "$@" > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o bench \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager "$@" > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o bench \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager "$@" > $OUT/write.log 2>&1
echo profile $TAG done
