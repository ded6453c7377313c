# step-level A/B of lab libraries: correctness of the touched module, then interleaved bench rounds
O=gpurun_out/${R:-r5m}
mkdir -p $O
for v in ${LIBS}; do
  [ "$v" = product ] && continue
  TGFR_LAB=1 TGFR_LIB=$GRAFT_REPO_ROOT/tools/lab/build/lib_$v.so timeout -k 10 300 python3 -u -m pytest ${TESTS} -x -q --timeout 120 --timeout-method thread > $O/test_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc: $(tail -1 $O/test_$v.log)"; [ $rc -le 1 ] || exit $rc
done
R=$R ROUNDS=${ROUNDS:-3} bash tools/lab/lib_ab.sh
