# round-6 GPU steps (run from the repo root on a GPU box): STEP selects
O=gpurun_out/${R:-r6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "${STEP:-trace}" in
trace)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 12
  tail -1 $O/trace.log | cut -c1-200
  ;;
envab)
  # interleaved A/B of environment settings: VARS="A=1 A=2 ..."
  for i in $(seq 1 ${ROUNDS:-3}); do
    for e in ${VARS}; do
      env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" ${BENCH_ARGS} > $O/bench_${e}_$i.log 2>&1 || exit 12
      echo "$e round $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${e}_$i.log | head -1)"
    done
  done
  ;;
esac
case "${STEP}" in
tracevars)
  for e in ${VARS}; do
    env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$e -o bench \
      -- python3 bench.py --steps 10 --warmup 3 --no-cpu --alt-precision "" > $O/trace_$e.log 2>&1 || exit 12
    echo "$e: $(grep -o '"ms_per_step": [0-9.]*' $O/trace_$e.log | head -1)"
  done
  ;;
esac
case "${STEP}" in
dp)
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dp.py tests/test_gpu_train.py -m gpu -v -s --timeout 600 --timeout-method thread > $O/dp.log 2>&1
  rc=$?; echo "dp tests rc=$rc: $(tail -1 $O/dp.log)"; [ $rc -le 1 ] || exit $rc
  timeout -k 10 240 python3 -u bench.py --simulate-world 8 --no-cpu --alt-precision "" > $O/sim8_cfg3.log 2>&1 || exit 22
  echo "sim8 cfg3: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_cfg3.log)"
  ;;
esac
case "${STEP}" in
dp2)
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dp.py -m gpu -v -s --timeout 600 --timeout-method thread -k "fp32-0-2" > $O/dp.log 2>&1
  echo "dp rc=$?: $(tail -1 $O/dp.log)"
  for i in 1 2 3; do for e in TGFR_TEXT_ASYNC=1 TGFR_TEXT_ASYNC=0; do
    env $e timeout -k 10 240 python3 -u bench.py --simulate-world 8 --no-cpu --alt-precision "" > $O/sim8_${e}_$i.log 2>&1 || exit 22
    echo "$e $i: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_${e}_$i.log)"
  done; done
  ;;
esac
case "${STEP}" in
qkv)
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tail.py tests/test_gpu_step_parity.py tests/test_gpu_modules.py tests/test_gpu_words.py -m gpu -v -s --timeout 200 --timeout-method thread -k "bn_qkv or imim or reduced or heading or image or bounded or seeded" > $O/qkv.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/qkv.log)"; [ $rc -le 1 ] || exit $rc
  for i in 1 2 3; do for e in TGFR_BN_QKV=1 TGFR_BN_QKV=0; do
    env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_${e}_$i.log 2>&1 || exit 22
    echo "$e $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${e}_$i.log)"
  done; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 12
  ;;
esac
case "${STEP}" in
qkv2)
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tail.py tests/test_gpu_step_parity.py tests/test_gpu_modules.py -m gpu -v -s --timeout 200 --timeout-method thread -k "bn_qkv or imim or reduced or heading or image" > $O/qkv.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/qkv.log)"; [ $rc -le 1 ] || exit $rc
  for i in 1 2 3; do for e in "TGFR_BN_QKV=1 TGFR_IMIM_PREP=1" "TGFR_BN_QKV=1 TGFR_IMIM_PREP=0" "TGFR_BN_QKV=0 TGFR_IMIM_PREP=0"; do
    t=$(echo $e | tr -d ' =_'); env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_${t}_$i.log 2>&1 || exit 22
    echo "$e $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${t}_$i.log)"
  done; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 12
  ;;
esac
case "${STEP}" in
lndw)
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_tail.py tests/test_abi.py -m gpu -v -s --timeout 200 --timeout-method thread > $O/lndw.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/lndw.log)"; [ $rc -le 1 ] || exit $rc
  for i in 1 2 3; do for e in TGFR_LN_DW_DEFER=1 TGFR_LN_DW_DEFER=0; do
    env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_${e}_$i.log 2>&1 || exit 22
    echo "$e $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${e}_$i.log)"
  done; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 12
  ;;
esac
case "${STEP}" in
quick)
  # TESTS="file::k ..." (pytest -k expression in KEXPR), then 3 benches and a trace
  timeout -k 10 600 python3 -u -m pytest ${TESTS} -m gpu -v -s --timeout 200 --timeout-method thread -k "${KEXPR}" > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -le 1 ] || exit $rc
  for i in 1 2 3; do
    timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_$i.log 2>&1 || exit 22
    echo "bench $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log)"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 12
  ;;
esac
case "${STEP}" in
cfg4fork)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_modules.py tests/test_gpu_dp.py tests/test_gpu_train.py -m gpu -v -s --timeout 300 --timeout-method thread -k "sent_global or identity or forked or dp_" > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -le 1 ] || exit $rc
  for e in TGFR_FORK=2 TGFR_FORK=0; do
    env $e timeout -k 10 300 python3 -u bench.py --batch 128 --words 64 --precision fp16 --simulate-world 8 --alt-precision "" > $O/sim8_cfg5_${e}.log 2>&1 || exit 22
    echo "$e sim8 cfg5: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_cfg5_${e}.log)"
  done
  timeout -k 10 240 python3 -u bench.py --simulate-world 8 --no-cpu --alt-precision "" > $O/sim8_cfg3.log 2>&1 || exit 23
  echo "sim8 cfg3: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_cfg3.log)"
  ;;
esac
case "${STEP}" in
order)
  for i in 1 2 3; do for e in ${VARS:-TGFR_ORDER=a TGFR_ORDER=g}; do
    env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_${e}_$i.log 2>&1 || exit 22
    echo "$e $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${e}_$i.log)"
  done; done
  TGFR_ORDER=${TRACE_ORDER:-g} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o bench \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 12
  ;;
esac
case "${STEP}" in
textpmc)
  P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
  P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/pmct1 -o t -- python3 tools/text_bench.py --reps 5 > $O/pmct1.log 2>&1 || exit 16
  timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $O/pmct2 -o t -- python3 tools/text_bench.py --reps 5 > $O/pmct2.log 2>&1 || exit 17
  echo textpmc ok
  ;;
esac
case "${STEP}" in
text)
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_text.py tests/test_gpu_step_parity.py -m gpu -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -le 1 ] || exit $rc
  timeout -k 10 120 python3 -u tools/text_bench.py > $O/text.log 2>&1 || exit 21
  grep "B=64" $O/text.log
  for i in 1 2 3; do
    timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_$i.log 2>&1 || exit 22
    echo "bench $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$i.log)"
  done
  ;;
esac
case "${STEP}" in
sim8prof)
  mkdir -p $O/prof_sim8
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sim8/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu --alt-precision "" --batch 128 --words 64 --precision fp16 --simulate-world 8 > $O/prof_sim8.trace.log 2>&1 || exit 13
  timeout -k 10 300 python3 -u bench.py --batch 128 --words 64 --precision fp16 --simulate-world 8 --alt-precision "" > $O/sim8_cfg5.log 2>&1 || exit 14
  echo "sim8 cfg5: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_cfg5.log)"
  ;;
esac
case "${STEP}" in
abtrace)
  # tests, interleaved bench A/B of VARS, then one kernel trace per variant
  timeout -k 10 600 python3 -u -m pytest ${TESTS} -m gpu -q --timeout 200 --timeout-method thread -k "${KEXPR}" > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -le 1 ] || exit $rc
  for i in 1 2 3; do for e in ${VARS}; do
    env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_${e}_$i.log 2>&1 || exit 22
    echo "$e $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${e}_$i.log)"
  done; done
  for e in ${VARS}; do
    env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$e -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace_$e.log 2>&1 || exit 12
  done
  ;;
esac
