# batching engines' decode-attention grid policy (batch-invariant candidates)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python scripts/microbench_kernels.py attn-rows > gpurun_out/r2_v8_attn_rows.log 2>&1
