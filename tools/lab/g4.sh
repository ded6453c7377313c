# full GPU suite + smoke + bench (one box)
O=gpurun_out/${R:-r5g}
mkdir -p $O
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 8
echo smoke ok
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -4 $O/gputest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python3 -u bench.py > $O/bench.log 2>&1 || exit 12
tail -1 $O/bench.log | cut -c1-300
