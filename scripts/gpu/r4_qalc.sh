# Round 4: qkv_attn attention chunk for long buckets on TP ranks: 256 vs 128 keys per block.
cd $GRAFT_REPO_ROOT
tag=${1:-r4qalc}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step c128 300 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,9000,17000 --tokens 256
step c256 300 env LLMC_QA_LONG_CHUNK=256 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,9000,17000 --tokens 256
step c128b 300 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,9000,17000 --tokens 256
