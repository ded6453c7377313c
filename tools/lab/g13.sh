# IMIM backward fork: IMIM / step tests with the fork on (default), then an
# interleaved config-2 step A/B of TGFR_IMIM_DW_FORK=0 / 1, then the FCFM
# (configs[3]) bench line
O=gpurun_out/${R:-r6i}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tail.py tests/test_gpu_step_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
R=${R:-r6i} ROUNDS=${ROUNDS:-3} ENVS="TGFR_IMIM_DW_FORK=0 TGFR_IMIM_DW_FORK=1" bash tools/lab/env_ab.sh || exit $?
timeout -k 10 300 python3 -u tools/fcfm_bench.py > $O/fcfm.log 2>&1 || exit 14
echo "fcfm: $(tail -1 $O/fcfm.log | cut -c1-200)"
