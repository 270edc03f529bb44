set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
(cd ab_head && timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1) > gpurun_out/r2_ab_head_bench.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/r2_ab_new_bench.log 2>&1 && \
(cd ab_head && timeout -k 10 400 python bench.py --gpus 1 --steps 2 --warmup 1) > gpurun_out/r2_ab_head_bench2.log 2>&1
