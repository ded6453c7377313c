O=gpurun_out/${R:-r5p}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_step_parity.py tests/test_gpu_words.py tests/test_gpu_text.py -q -s --timeout 300 --timeout-method thread > $O/tol.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 $O/tol.log
