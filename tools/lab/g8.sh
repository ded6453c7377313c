# per-rank simulate-world-8 profiles (trace + FETCH/WRITE) of configs[2] and configs[4]
O=gpurun_out/${R:-r5o}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {   # prof <dir> <bench args...>
  local D=$O/$1; shift
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision "" "$@" > $D.trace.log 2>&1 || return 13
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $D/fetch -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager "$@" > $D.fetch.log 2>&1 || return 14
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $D/write -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu --alt-precision "" --eager "$@" > $D.write.log 2>&1 || return 15
}
timeout -k 10 240 python3 -u bench.py --batch 64 --simulate-world 8 --no-cpu --alt-precision "" > $O/sim8_cfg3.json.log 2>&1 || exit 11
echo "cfg3 sim8: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_cfg3.json.log)"
prof prof_sim8_cfg3 --batch 64 --simulate-world 8 || exit $?
echo prof cfg3 ok
timeout -k 10 300 python3 -u bench.py --batch 128 --words 64 --precision fp16 --simulate-world 8 --no-cpu --alt-precision "" > $O/sim8_cfg5.json.log 2>&1 || exit 16
echo "cfg5 sim8: $(grep -o '"ms_per_step": [0-9.]*' $O/sim8_cfg5.json.log)"
prof prof_sim8_cfg5 --batch 128 --words 64 --precision fp16 --simulate-world 8 || exit $?
echo prof cfg5 ok
