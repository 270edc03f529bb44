# Per-rank decode evidence for BASELINE configs 4/5 and the N=8 judge: one
# tensor-parallel rank's shard alone on one GPU (no all-reduces), plus the whole Mixtral / Phi-3
# responders, each under rocprofv3 kernel stats.
# usage: gpurun --timeout 1100 -- bash scripts/gpu/shards.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=${1:-sh}
mkdir -p gpurun_out
bash scripts/prof_tp_shard.sh ${tag}_70b_tp4 --model llama-3-70b --tp 4 --ctx 2048,16384 --tokens 256 && \
bash scripts/prof_tp_shard.sh ${tag}_70b_tp2 --model llama-3-70b --tp 2 --ctx 2048,16384 --tokens 256 && \
bash scripts/prof_tp_shard.sh ${tag}_8b_tp8 --model llama-3-8b --tp 8 --ctx 2048,33000 --tokens 256 && \
bash scripts/prof_decode.sh ${tag}_mixtral_2k --model mixtral-8x7b --prompt 2048 --ctx 4096 --tokens 256 && \
bash scripts/prof_decode.sh ${tag}_phi3_2k --model phi-3-mini --prompt 2048 --ctx 4096 --tokens 256
