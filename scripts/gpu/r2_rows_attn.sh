# row-aware attention buckets for batching engines: engine/batcher tests, decode steps, serving
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_batcher.py tests/test_server.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_rows_attn_tests.log 2>&1 && \
rm -f gpurun_out/r2_rows_steps.log && \
for b in 4 16; do timeout -k 10 300 python -u scripts/profile_decode.py --batch $b --tokens 512 --prompt 2000 >> gpurun_out/r2_rows_steps.log 2>&1 || exit 1; done && \
timeout -k 10 900 python -u scripts/serve_bench.py --concurrency 4,16 --requests 16 --max-tokens 512 > gpurun_out/r2_rows_serve.log 2>&1
