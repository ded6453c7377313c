O=gpurun_out/r5d
mkdir -p $O
TGFR_LAB=1 TGFR_LIB=$GRAFT_REPO_ROOT/tools/lab/build/lib_stamp.so timeout -k 10 120 python3 -u true

LAB_ROUNDS=3 timeout -k 10 400 python3 -u tools/lab/bench_variants.py > $O/lab.log 2>&1 || exit 9
cat $O/lab.log
