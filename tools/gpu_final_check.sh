# Final check of the tree as committed (run from the repo root on a GPU box):
# smoke(), the whole GPU suite, the default bench line and configs[4]'s
# caption length at N = 1.  Every step has its own limit; stops at a failure.
O=gpurun_out/${R:-final}
mkdir -p $O
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 8
echo smoke ok
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc: $(tail -1 $O/gputest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 -u bench.py > $O/bench.log 2>&1 || exit 12
echo "bench: $(tail -1 $O/bench.log | cut -c1-220)"
timeout -k 10 240 python3 -u bench.py --batch 128 --words 64 --precision fp16 --no-cpu --alt-precision "" > $O/bench_cfg5.log 2>&1 || exit 13
echo "cfg5: $(tail -1 $O/bench_cfg5.log | cut -c1-220)"
