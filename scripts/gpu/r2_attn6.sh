set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "attn_decode or engine or logits or prefill" -x -q --timeout 200 --timeout-method thread > gpurun_out/r2_attn6_tests.log 2>&1 && \
timeout -k 10 500 python scripts/microbench_kernels.py attn > gpurun_out/r2_attn6_micro.log 2>&1 && \
timeout -k 10 300 python scripts/tp_shard_decode.py --tp 1,2,4,8 --ctx 2048,33000 > gpurun_out/r2_attn6_shards.log 2>&1 && \
timeout -k 10 300 python scripts/tp_shard_decode.py --model llama-3-70b --tp 4,8 --ctx 2048,16384 > gpurun_out/r2_attn6_shards70.log 2>&1
