set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/microbench_kernels.py gemm-ab > gpurun_out/r2_gemm_ab.log 2>&1
