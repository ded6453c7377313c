set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export TGFR_GEMM_CFG=0
P="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc1 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pmc1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc2 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pmc2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc3 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pmc3.log 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc4 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pmc4.log 2>&1
