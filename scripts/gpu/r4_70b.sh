# Round 4: Llama-3-70B TP=4 / TP=8 rank shards with the one-launch qkv + attention (all) vs two launches.
cd $GRAFT_REPO_ROOT
tag=${1:-r4_70b}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step qa 400 env LLMC_QKV_ATTN=all python -u scripts/tp_shard_decode.py --model llama-3-70b --tp 8,4 --ctx 2048,16000 --tokens 128
step off 400 env LLMC_QKV_ATTN=0 python -u scripts/tp_shard_decode.py --model llama-3-70b --tp 8,4 --ctx 2048,16000 --tokens 128
