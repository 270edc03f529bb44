# rocprofv3 kernel stats of batch-1 decode: Llama-3-8B at 2k and 13.5k context, a TP=8 rank's
# shard at 2k and 33k (profiles/<tag>_*). usage: gpurun -- bash scripts/gpu/profile_decode.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-dec}
mkdir -p gpurun_out
bash scripts/prof_decode.sh ${tag}_8b_2k --prompt 2048 --ctx 8192 --tokens 512 && \
bash scripts/prof_decode.sh ${tag}_8b_13k --prompt 13500 --ctx 20480 --tokens 512 && \
bash scripts/prof_tp_shard.sh ${tag}_tp8_2k --tp 8 --ctx 2048 --tokens 512 && \
bash scripts/prof_tp_shard.sh ${tag}_tp8_33k --tp 8 --ctx 33000 --tokens 512
