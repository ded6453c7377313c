# config-2 step A/B (HEAD vs work tree) after the touched modules' GPU tests
O=gpurun_out/${R:-r6e}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_words.py tests/test_gpu_tail.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
R=${R:-r6e} ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-head product}" bash tools/lab/lib_ab.sh
