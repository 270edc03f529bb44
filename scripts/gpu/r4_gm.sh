# Round 4: prefill GEMM grouped tile order, M-tiles per group 4 / 8 (default) / 16 / 32.
cd $GRAFT_REPO_ROOT
tag=${1:-r4gm}
mkdir -p gpurun_out
source scripts/gpu/steps.sh
for g in 8 4 16 32 8; do
  step gm$g 240 env LLMC_GEMM_GROUP_M=$g python -u scripts/microbench_kernels.py prefill
done
