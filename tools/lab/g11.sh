# T=64 forward: words tests on the product, res2 stamps, interleaved bench A/B (HEAD vs work tree)
O=gpurun_out/${R:-r6a}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_words.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/test_words.log 2>&1
rc=$?; echo "words tests rc=$rc: $(tail -1 $O/test_words.log)"; [ $rc -eq 0 ] || exit $rc
if [ -f tools/lab/build/lib_rstamp.so ]; then
  TGFR_LAB=1 TGFR_LIB=$GRAFT_REPO_ROOT/tools/lab/build/lib_rstamp.so timeout -k 10 150 python3 tools/lab/rstamps.py > $O/rstamps.log 2>&1 || exit 11
fi
R=${R:-r6a} ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-head product}" BENCH_ARGS="${BENCH_ARGS:---batch 128 --words 64 --precision fp16}" bash tools/lab/lib_ab.sh
