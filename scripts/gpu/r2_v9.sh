# batching engines' length-only attention split (min 2048 keys per block): tests, a lone long row
# and full batches on a 32-row serving engine, serving throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_batcher.py tests/test_engine_gpu.py tests/test_server.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r2_v9_tests.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --batch 1 --engine-rows 32 --prompt 13500 --ctx 16384 --tokens 256 > gpurun_out/r2_v9_lone.log 2>&1 && \
timeout -k 10 200 python scripts/profile_decode.py --batch 1 --prompt 13500 --ctx 16384 --tokens 256 >> gpurun_out/r2_v9_lone.log 2>&1 && \
timeout -k 10 300 python scripts/profile_decode.py --batch 16 --prompt 2500 --ctx 4096 --tokens 256 > gpurun_out/r2_v9_rows.log 2>&1 && \
timeout -k 10 300 python scripts/profile_decode.py --batch 32 --prompt 2500 --ctx 4096 --tokens 256 >> gpurun_out/r2_v9_rows.log 2>&1 && \
timeout -k 10 600 python -u scripts/serve_bench.py --concurrency 1,16,32 --requests 32 --max-tokens 512 > gpurun_out/r2_v9_serve.log 2>&1
