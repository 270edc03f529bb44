# Round 4: qkv_attn with one sentinel poller per block: its tests and the TP shard A/B over contexts.
cd $GRAFT_REPO_ROOT
tag=${1:-r4qa2}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tests 300 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 200 --timeout-method thread
step qa8 300 python -u scripts/tp_shard_decode.py --tp 8 --ctx 2048,4096,8192,12000,16000,20000 --tokens 256
step tl8 300 env LLMC_QKV_ATTN=0 python -u scripts/tp_shard_decode.py --tp 8 --ctx 2048,4096,8192,12000,16000,20000 --tokens 256
step qa4 300 python -u scripts/tp_shard_decode.py --tp 4 --ctx 2048,6000,10500 --tokens 256
step tl4 300 env LLMC_QKV_ATTN=0 python -u scripts/tp_shard_decode.py --tp 4 --ctx 2048,6000,10500 --tokens 256
