# Round 4: decode-attention counters one 128-B line per word: attention tests, attention
# microbenchmarks (8B and TP-rank head counts), 8B decode at ~9k and the TP=8 shard at 2k.
# usage: gpurun --timeout 900 -- bash scripts/gpu/r4_ctr.sh <tag>
cd $GRAFT_REPO_ROOT
tag=${1:-r4ctr}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attn_oproj_gpu.py tests/test_engine_gpu.py -x -q -k "attn or decode" --timeout 200 --timeout-method thread
step attn 300 python -u scripts/microbench_kernels.py attn
step attn_tp 300 python -u scripts/microbench_kernels.py attn-tp
step dec9k 300 bash scripts/prof_decode.sh ${tag}_dec9k --prompt 8704 --ctx 9400 --tokens 512
step shard 200 python -u scripts/tp_shard_decode.py --tp 8 --ctx 2048 --tokens 256
step shard20k 200 python -u scripts/tp_shard_decode.py --tp 8 --ctx 20000 --tokens 256
