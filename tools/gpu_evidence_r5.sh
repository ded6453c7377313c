# Round-5 evidence, two GPU calls (run from the repo root on a GPU box):
#   PART=1: tools/gpu_evidence.sh with SIM8=1 -- smoke, GPU tests, the default
#           bench line, config-2 trace + FETCH/WRITE passes, SQ passes,
#           configs[4] per-rank trace + passes;
#   PART=2: the bench lines of the other shapes -- configs[4]'s caption
#           length at N = 1 (B = 128, T = 62, fp16) and the simulate-world-8
#           per-rank steps of configs[2] and configs[4].
R=${R:-r5e}
O=gpurun_out/$R
mkdir -p $O
if [ "${PART:-1}" = 1 ]; then
  SIM8=1 R=$R bash tools/gpu_evidence.sh || exit $?
  exit 0
fi
timeout -k 10 240 python3 -u bench.py --batch 128 --words 64 --precision fp16 --no-cpu > $O/bench_cfg5_shape.log 2>&1 || exit 21
echo cfg5 shape ok
timeout -k 10 240 python3 -u bench.py --simulate-world 8 --no-cpu --alt-precision "" > $O/bench_sim8_cfg3.log 2>&1 || exit 22
echo sim8 cfg3 ok
timeout -k 10 300 python3 -u bench.py --batch 128 --words 64 --precision fp16 --simulate-world 8 --no-cpu --alt-precision "" > $O/bench_sim8_cfg5.log 2>&1 || exit 23
echo sim8 cfg5 ok
