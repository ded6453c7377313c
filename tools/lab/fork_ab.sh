# A/B of the single-process step with the g' branch forked onto a side stream
# (TGFR_FORK=1, the default) against the linear graph (TGFR_FORK=0): the step's
# parity tests on the fork path first, then interleaved bench lines.
O=gpurun_out/${R:-fork}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step_parity.py tests/test_gpu_dp.py -q -x --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 1
echo parity ok
for i in 1 2; do
  for f in ${FORKS:-0 1}; do
    TGFR_FORK=$f timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_fork${f}_$i.log 2>&1 || exit 12
    echo "fork=$f round $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_fork${f}_$i.log)"
  done
done
