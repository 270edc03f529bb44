# Round 4: one-engine decode at 2k (TP=1 shard timing, as profiles/r3_shard_timings.log) and the engine
# bench with 3 timed rounds, to separate kernel changes from box-to-box variance.
cd $GRAFT_REPO_ROOT
tag=${1:-r4ab}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
step shard1 200 python -u scripts/tp_shard_decode.py --tp 1 --ctx 2048 --tokens 256
step gemv 200 python -u scripts/microbench_kernels.py gemv
step bench 330 python -u bench.py --steps 3 --warmup 1
