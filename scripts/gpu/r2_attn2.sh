set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "attn" -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_attn2_tests.log 2>&1 && \
timeout -k 10 300 python scripts/microbench_kernels.py attn > gpurun_out/r2_attn2_microbench.log 2>&1
