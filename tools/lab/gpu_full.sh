# One GPU call: word<->region parity first; the lab A/B; then (parity green)
# the whole GPU suite, the bench line and the round's rocprofv3 evidence.
R=${R:-r4x}
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_words.py -q --timeout 120 --timeout-method thread -x > $O/words.log 2>&1
rc=$?
echo "words rc=$rc"
[ $rc -le 1 ] || exit $rc
LAB_ROUNDS=${LAB_ROUNDS:-3} timeout -k 10 400 python3 -u tools/lab/bench_variants.py > $O/lab.log 2>&1 || exit 9
echo lab ok
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
echo "gputest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 python3 -u bench.py > $O/bench.log 2>&1 || exit 12
echo bench ok
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/trace.log 2>&1 || exit 13
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager > $O/fetch.log 2>&1 || exit 14
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager > $O/write.log 2>&1 || exit 15
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/pmcw1 -o w -- python3 tools/microbench.py --bf16-only 64 > $O/pmcw1.log 2>&1 || exit 16
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $O/pmcw2 -o w -- python3 tools/microbench.py --bf16-only 64 > $O/pmcw2.log 2>&1 || exit 17
echo profile ok
