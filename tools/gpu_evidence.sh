# One GPU call for a round's evidence (run from the repo root on a GPU box):
#   1. the GPU tests of FIRST (default: the module tests), then the whole GPU suite
#   2. the default bench line
#   3. rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of the bench
#      configuration (tools/profile_round.sh layout: prof_<R>_cfg2)
#   4. SQ counter passes of the word<->region kernels (tools/microbench.py)
#   5. (SIM8=1) the same trace / PMC passes for configs[4]'s per-rank step
#      (B = 128, T = 62, fp16, --simulate-world 8): prof_<R>_sim8
# PROF=trace: the kernel trace only; SQ=0: no SQ passes (and no SIM8);
# LAB=1: tools/lab/bench_variants.py after the first tests.
# Every GPU step has its own time limit; the script stops at the first
# failure.  Summaries: tools/summarize_profile.py / tools/summarize_sq.py here.
R=${R:-r4x}
O=gpurun_out/$R
FIRST=${FIRST:-tests/test_gpu_modules.py}
mkdir -p $O
timeout -k 10 180 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 8
echo smoke ok
timeout -k 10 300 python3 -u -m pytest $FIRST -q -x --timeout 120 --timeout-method thread > $O/first.log 2>&1
rc=$?; echo "first rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ "${LAB:-0}" = 1 ]; then     # A/B of the lab variants in tools/lab/build
  LAB_ROUNDS=${LAB_ROUNDS:-3} timeout -k 10 400 python3 -u tools/lab/bench_variants.py > $O/lab.log 2>&1 || exit 9
  echo lab ok
fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 180 python3 -u bench.py > $O/bench.log 2>&1 || exit 12
echo bench ok
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {   # prof <dir> <bench args...>
  local D=$O/$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" "$@" > $D.trace.log 2>&1 || return 13
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $D/fetch -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager "$@" > $D.fetch.log 2>&1 || return 14
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $D/write -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager "$@" > $D.write.log 2>&1 || return 15
}
if [ "${PROF:-1}" = 1 ]; then
  mkdir -p $O/prof_cfg2
  prof prof_cfg2 || exit $?
  echo profile cfg2 ok
elif [ "${PROF:-1}" = trace ]; then
  mkdir -p $O/prof_cfg2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg2/trace -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" > $O/prof_cfg2.trace.log 2>&1 || exit 13
  echo trace cfg2 ok
fi
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
[ "${SQ:-1}" = 1 ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/pmcw1 -o w -- python3 tools/microbench.py --bf16-only 64 > $O/pmcw1.log 2>&1 || exit 16
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $O/pmcw2 -o w -- python3 tools/microbench.py --bf16-only 64 > $O/pmcw2.log 2>&1 || exit 17
echo sq ok
if [ "${SIM8:-0}" = 1 ]; then
  mkdir -p $O/prof_sim8
  prof prof_sim8 --batch 128 --words 64 --precision fp16 --simulate-world 8 || exit $?
  echo profile sim8 ok
fi
