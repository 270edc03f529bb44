# Round 4: where a TP=8 rank's decode layer goes: launch floor, decode attention at the TP ranks'
# head counts (fused / split grids), rocprofv3 kernel table of the 8B TP=8 shard at 2k, per-layer
# numerics at the judge context.
# usage: gpurun --timeout 900 -- bash scripts/gpu/r4_tp.sh <tag>
cd $GRAFT_REPO_ROOT
tag=${1:-r4tp}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step launch 120 python -u scripts/microbench_kernels.py launch
step attn_tp 300 python -u scripts/microbench_kernels.py attn-tp
step shard_prof 300 bash scripts/prof_tp_shard.sh ${tag}_shard8 --tp 8 --ctx 2048 --tokens 256
step perlayer 300 python -u -m pytest tests/test_numerics_full_gpu.py -k per_layer -x -q -s --timeout 280 --timeout-method thread
