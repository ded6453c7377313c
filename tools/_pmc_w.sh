set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
timeout -k 10 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pw1 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pw1.log 2>&1
timeout -k 10 60 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pw2 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pw2.log 2>&1
TGFR_GEMM_WRES=0 timeout -k 10 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pw3 -o g -- python3 tools/gemm_one.py qkv_fwd 5 > gpurun_out/pw3.log 2>&1
