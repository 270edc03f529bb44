set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python scripts/microbench_kernels.py attn > gpurun_out/r2_attn_all.log 2>&1
