# Kernel microbenchmarks (scripts/microbench_kernels.py: prefill | attn | moe | ...).
# usage: gpurun -- bash scripts/gpu/microbench.sh <tag> <which>...
set -o pipefail
cd $GRAFT_REPO_ROOT
tag=$1; shift
mkdir -p gpurun_out
for w in "$@"; do
  timeout -k 10 300 python scripts/microbench_kernels.py $w > gpurun_out/${tag}_${w}.log 2>&1 || exit $?
done
