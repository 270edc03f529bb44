# rocprofv3 kernel stats of one bench round at the default shape (3 x 8B responders + 8B judge on
# one GPU). usage: gpurun -- bash scripts/gpu/profile_bench.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/prof_bench.sh ${1:-bench}_prof --steps 1 --warmup 1
