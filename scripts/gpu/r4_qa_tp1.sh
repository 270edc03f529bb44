# Round 4: where the one-launch qkv + attention loses on the whole 8B (TP=1): rocprofv3 tables with
# it on every bucket vs the two launches (attn_oproj off in both), 2k keys.
cd $GRAFT_REPO_ROOT
tag=${1:-r4qa1}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
export LLMC_ATTN_OPROJ=0
step on 300 env LLMC_QKV_ATTN=all bash scripts/prof_tp_shard.sh ${tag}_on --tp 1 --ctx 2048 --tokens 256
step off 300 env LLMC_QKV_ATTN=0 bash scripts/prof_tp_shard.sh ${tag}_off --tp 1 --ctx 2048 --tokens 256
