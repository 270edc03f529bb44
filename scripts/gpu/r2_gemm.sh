set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gemm_tests.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py prefill > gpurun_out/r2_gemm_microbench.log 2>&1
