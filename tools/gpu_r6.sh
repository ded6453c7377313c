O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_words.py tests/test_gpu_step_parity.py -m gpu -v -s --timeout 200 --timeout-method thread -k "fp16 or captured or seeded or reduced" > $O/words.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/words.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --no-cpu > $O/bench.log 2>&1 || exit 12
echo "bench: $(tail -1 $O/bench.log | cut -c1-400)"
