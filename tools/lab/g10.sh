# T=64 backward: words tests on the product, then interleaved bench A/B at configs[5]'s rank shape
O=gpurun_out/${R:-r5w}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_words.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/test_words.log 2>&1
rc=$?; echo "words tests rc=$rc: $(tail -1 $O/test_words.log)"; [ $rc -eq 0 ] || exit $rc
R=${R:-r5w} ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-burst product nopha}" BENCH_ARGS="${BENCH_ARGS:---batch 128 --words 64 --precision fp16}" bash tools/lab/lib_ab.sh
