# Round 4: segment-ordered qkv_attn on every shape: tests, shard A/B at TP=1 / 2 / 4 / 8
# (LLMC_QKV_ATTN=all vs 0), then the one-GPU bench with all vs default.
cd $GRAFT_REPO_ROOT
tag=${1:-r4qa4}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tests 400 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 200 --timeout-method thread
step all 400 env LLMC_QKV_ATTN=all python -u scripts/tp_shard_decode.py --tp 1,2,4,8 --ctx 2048,7500,9000 --tokens 256
step off 400 env LLMC_QKV_ATTN=0 python -u scripts/tp_shard_decode.py --tp 1,2,4,8 --ctx 2048,7500,9000 --tokens 256
