# Round 4: qkv_attn with the o_proj role: tests, TP suites, shard A/B (LLMC_QKV_ATTN_O=1 vs 0),
# the TP=8-shaped rehearsal over 2 CU-partitioned ranks (fused all-reduce in the o_proj role).
cd $GRAFT_REPO_ROOT
tag=${1:-r4qao}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step tests 400 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 200 --timeout-method thread
step tests2 500 python -u -m pytest tests/test_tp_gpu.py tests/test_engine_gpu.py tests/test_custom_ar_gpu.py -x -q --timeout 200 --timeout-method thread
step o1 300 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,9000,20000 --tokens 256
step o0 300 env LLMC_QKV_ATTN_O=0 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,9000,20000 --tokens 256
step reh1 200 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 1
step reh0 200 env LLMC_QKV_ATTN_O=0 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 1
