O=gpurun_out/${R:-r5h}
mkdir -p $O
true




LAB_ROUNDS=3 timeout -k 10 400 python3 -u tools/lab/bench_variants.py > $O/lab.log 2>&1 || exit 9
grep SUMMARY $O/lab.log
