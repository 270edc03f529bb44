# batched-decode (MFMA form) numerics + microbenchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemvm or batched or qkv_rope or fused_norm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_gemvm_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_gemvm_engine.log 2>&1 && \
timeout -k 10 300 python -u scripts/microbench_kernels.py batched > gpurun_out/r2_gemvm_bench.log 2>&1
