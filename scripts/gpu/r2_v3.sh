set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --steps 3 --warmup 2 > gpurun_out/r2_v3_bench.log 2>&1 && \
bash scripts/prof_bench.sh r2_v3_prof --steps 1 --warmup 0 --max-tokens 1024
