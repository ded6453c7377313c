set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for shape in qkv_fwd attn_s; do
timeout -k 10 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --kernel-trace --output-format csv -d gpurun_out/pg_$shape -o g -- python3 tools/gemm_one.py $shape 5 > gpurun_out/pg_$shape.log 2>&1
timeout -k 10 60 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d gpurun_out/pt_$shape -o g -- python3 tools/gemm_one.py $shape 5 > gpurun_out/pt_$shape.log 2>&1
done
