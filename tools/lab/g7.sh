O=gpurun_out/${R:-r5n}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_dp.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $O/dp.log 2>&1
rc=$?; echo "dp rc=$rc"; tail -5 $O/dp.log
[ $rc -le 1 ] || exit $rc
for f in 0 2; do
  TGFR_FORK=$f timeout -k 10 240 python3 -u bench.py --batch 64 --simulate-world 8 --no-cpu --alt-precision "" > $O/sim8_fork$f.log 2>&1 || exit 12
  echo "fork $f: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_fork$f.log)"
done
