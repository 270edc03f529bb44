# Round 4 final validation after the last qkv_attn change: GPU test suite, smoke, TP shards, rehearsal.
cd $GRAFT_REPO_ROOT
tag=${1:-r4fin2}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step pytest 600 python -u -m pytest tests/ -m gpu -q -rs --timeout 200 --timeout-method thread
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
step shard 300 python -u scripts/tp_shard_decode.py --tp 8,4 --ctx 2048,17000 --tokens 256
step reh 200 python -u scripts/tp_rehearsal.py --shape-tp 8 --world 2 --fused-ar 1
