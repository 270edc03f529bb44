# Round 4: one-launch qkv + attention for the TP ranks' shards (csrc/kernels/qkv_attn.hip): its tests,
# the engine / TP tests that now run it (llama-small), and the shard decode A/B (LLMC_QKV_ATTN=0/1).
cd $GRAFT_REPO_ROOT
tag=${1:-r4qa}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tests 400 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 200 --timeout-method thread
step tests2 500 python -u -m pytest tests/test_engine_gpu.py tests/test_tp_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread
step shard_qa 300 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,20000 --tokens 256
step shard_2l 300 env LLMC_QKV_ATTN=0 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,20000 --tokens 256
