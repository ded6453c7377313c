#!/bin/bash
# tail tests, then a kernel trace of the default bench (graph replay) into gpurun_out/$1
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tr}
rm -rf $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_tail.py} > gpurun_out/${1:-tr}_tests.log 2>&1
tail -2 gpurun_out/${1:-tr}_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $OUT.log 2>&1
grep -o '"value": [0-9.]*, "unit": "pairs/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' $OUT.log
