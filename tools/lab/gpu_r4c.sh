mkdir -p gpurun_out/r4c
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_words.py -q --timeout 120 --timeout-method thread -x > gpurun_out/r4c/words.log 2>&1
rc=$?
echo "words rc=$rc"
if [ $rc -le 1 ]; then
  LAB_ROUNDS=3 timeout -k 10 300 python3 -u tools/lab/bench_variants.py > gpurun_out/r4c/lab.log 2>&1 && echo lab ok && \
  timeout -k 10 120 python3 -u bench.py > gpurun_out/r4c/bench.log 2>&1 && echo bench ok
fi
