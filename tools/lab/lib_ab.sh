# Interleaved bench A/B of lab builds of the library (tools/lab/variants.py
# FILE_VARIANTS): LIBS lists variant names ("product" = the in-tree library);
# ROUNDS rounds each.
O=gpurun_out/${R:-libab}/ab
mkdir -p $O
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in ${LIBS}; do
    if [ "$v" = product ]; then L=""; else L=$GRAFT_REPO_ROOT/tools/lab/build/lib_$v.so; fi
    TGFR_LAB=1 TGFR_LIB=$L timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" ${BENCH_ARGS} > $O/bench_${v}_$i.log 2>&1 || exit 12
    echo "$v round $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$i.log)"
  done
done
