# Prefill GEMM check: kernel tests, then the prefill microbench (ours vs hipBLASLt).
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-gemm}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or moe" -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/microbench_kernels.py prefill > gpurun_out/${tag}_prefill.log 2>&1
