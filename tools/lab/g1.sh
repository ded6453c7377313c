O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_words.py -x -q -s --timeout 120 --timeout-method thread > $O/words.log 2>&1
rc=$?; echo "words rc=$rc"; tail -5 $O/words.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -u tools/microbench.py --bf16-only 64 > $O/mb.log 2>&1 || exit 11
cat $O/mb.log
timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench.log 2>&1 || exit 12
tail -1 $O/bench.log | cut -c1-400
