# Round 4: rocprofv3 kernel table of the TP=8 and TP=4 shards with the one-launch qkv + attention.
cd $GRAFT_REPO_ROOT
tag=${1:-r4qa3}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step prof8 300 bash scripts/prof_tp_shard.sh ${tag}_tp8 --tp 8 --ctx 2048 --tokens 256
step prof8l 300 bash scripts/prof_tp_shard.sh ${tag}_tp8_20k --tp 8 --ctx 20000 --tokens 256
step tests 600 python -u -m pytest tests/test_tp_gpu.py tests/test_multigpu_gpu.py tests/test_custom_ar_gpu.py tests/test_bench_gpu.py -x -q -rs --timeout 200 --timeout-method thread
