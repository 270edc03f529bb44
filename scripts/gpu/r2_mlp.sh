set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "mlp_fused" -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_mlp_tests.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py mlp > gpurun_out/r2_mlp_micro.log 2>&1
