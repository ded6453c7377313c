set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
timeout -k 10 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pa1 -o g -- python3 tools/arc_one.py > gpurun_out/pa1.log 2>&1
timeout -k 10 60 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT --kernel-trace --output-format csv -d gpurun_out/pa2 -o g -- python3 tools/arc_one.py > gpurun_out/pa2.log 2>&1
