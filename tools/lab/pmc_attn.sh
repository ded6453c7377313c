# SQ counter passes for the fused attention kernels (attn_ablate.py base)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
python3 tools/lab/attn_ablate.py base > /dev/null
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmca1 -o a -- python3 tools/lab/attn_ablate.py base > gpurun_out/pmca1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d gpurun_out/pmca2 -o a -- python3 tools/lab/attn_ablate.py base > gpurun_out/pmca2.log 2>&1
echo pmc ok
