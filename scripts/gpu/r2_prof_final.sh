# rocprofv3 kernel stats of one bench round (3 x 8B responders + 8B judge, 1024 tokens each) on the final round-2 tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/prof_bench.sh r2_final_prof --steps 1 --warmup 0 --max-tokens 1024
