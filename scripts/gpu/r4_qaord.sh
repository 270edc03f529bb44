# Round 4: qkv_attn block order A/B on the TP=4 / TP=8 shards: per-head segments (shipped) vs every
# GEMV block first.
cd $GRAFT_REPO_ROOT
tag=${1:-r4qaord}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step seg 300 python -u scripts/tp_shard_decode.py --tp 4,8 --ctx 2048,9000,17000 --tokens 256
step gf 300 env LLMC_QA_ORDER=gemv_first python -u scripts/tp_shard_decode.py --tp 4,8 --ctx 2048,9000,17000 --tokens 256
step seg2 300 python -u scripts/tp_shard_decode.py --tp 4,8 --ctx 2048,9000,17000 --tokens 256
step gf2 300 env LLMC_QA_ORDER=gemv_first python -u scripts/tp_shard_decode.py --tp 4,8 --ctx 2048,9000,17000 --tokens 256
