set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/microbench_kernels.py attn-tp > gpurun_out/r2_attn_tp.log 2>&1
