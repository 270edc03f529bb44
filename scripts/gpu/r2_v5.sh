# 17-32-row MFMA decode form: kernel + engine tests, microbench vs 16 rows, serving at 32 requests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemvm or linear_batched or qkv_rope or batched_decode_rows" > gpurun_out/r2_v5_tests.log 2>&1 && \
timeout -k 10 400 python scripts/microbench_kernels.py batched32 > gpurun_out/r2_v5_micro.log 2>&1 && \
timeout -k 10 600 python -u scripts/serve_bench.py --concurrency 16,32 --requests 32 --max-tokens 512 > gpurun_out/r2_v5_serve.log 2>&1
