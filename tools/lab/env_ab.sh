# Interleaved bench A/B of environment switches (one box): ENVS lists the
# settings, e.g. ENVS="TGFR_AUX=0 TGFR_AUX=1"; ROUNDS rounds each.
O=gpurun_out/${R:-envab}
mkdir -p $O
for i in $(seq 1 ${ROUNDS:-2}); do
  for e in ${ENVS}; do
    env $e timeout -k 10 180 python3 -u bench.py --no-cpu --alt-precision "" > $O/bench_${e}_$i.log 2>&1 || exit 12
    echo "$e round $i: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${e}_$i.log)"
  done
done
